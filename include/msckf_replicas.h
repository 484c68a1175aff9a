/*
 * msckf_replicas.h -- C-ABI of the multi-GPU replica transport (RCCL over
 * xGMI), part of libmsckf_hip.so.
 *
 * The reference has no collectives: its only concurrency is the producer /
 * consumer threads of the VIO harness (MSCKF/vio.py:23-28).  The MI355X
 * throughput runs shard independent filters (or sequences) one process per
 * GPU (BASELINE north star: "via RCCL over xGMI ... the filter
 * itself has no cross-GPU collectives"), so RCCL carries control only: the
 * start / stop barriers of a timed region, the max over ranks of its elapsed
 * time and the gather of each rank's device identity.  Nothing on the filter
 * data path crosses GPUs.
 *
 * librccl is opened at run time (dlopen) by msckf_rccl_unique_id /
 * msckf_rccl_init, so the filter library does not depend on it.
 * Conventions as msckf_hip.h: 0 on success, < 0 on error,
 * msckf_rccl_last_error() for the message.
 */
#ifndef MSCKF_REPLICAS_H
#define MSCKF_REPLICAS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSCKF_RCCL_ID_BYTES 128

typedef struct msckf_rccl msckf_rccl_t;

/* ncclGetUniqueId: rank 0 creates the id and hands it to the other ranks out
 * of band (the replicas' TCP hub). */
int msckf_rccl_unique_id(uint8_t* id_out /* MSCKF_RCCL_ID_BYTES */);
/* ncclCommInitRankConfig on HIP device hip_device, non-blocking: gives up
 * (ncclCommAbort, returns -4) if the communicator is not ready within
 * timeout_s seconds, so a launcher can fall back to its host transport. */
int msckf_rccl_init(const uint8_t* id, int nranks, int rank, int hip_device, double timeout_s,
                    msckf_rccl_t** out);
/* In-place all-reduce of n doubles (op 0 = sum, 1 = max) through device
 * memory on the communicator's stream; returns after the stream synchronises
 * (a barrier when n = 1). */
int msckf_rccl_allreduce(msckf_rccl_t* c, double* v, int n, int op);
/* All-gather of nbytes per rank: all_out receives nranks * nbytes, rank order. */
int msckf_rccl_allgather(msckf_rccl_t* c, const void* mine, int nbytes, void* all_out);
/* Deadline (seconds) of every later wait on this communicator: collectives
 * and the teardown.  A launcher whose ranks do unequal work between two
 * collectives (rank 0's accuracy / ATE legs) sets it generously. */
int msckf_rccl_set_timeout(msckf_rccl_t* c, double timeout_s);
/* ncclCommCount (ranks in the communicator) and the communicator's rank. */
int msckf_rccl_count(const msckf_rccl_t* c, int* count_out, int* rank_out);
/* ncclCommFinalize, polled to completion, then ncclCommDestroy; a teardown
 * that fails or outlives the deadline is aborted (returns -4). */
int msckf_rccl_destroy(msckf_rccl_t* c);
const char* msckf_rccl_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MSCKF_REPLICAS_H */
