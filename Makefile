# Builds the HIP extension in-tree for gfx950 (the .so travels to the GPU box
# with the gpurun snapshot; it is git-ignored).
PKG      := visual-inertial-odometry-msckf-stereo_amd
SRC      := $(PKG)/csrc
LIB      := $(PKG)/libmsckf_hip.so
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) --offload-compress -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -Iinclude -fno-slp-vectorize
OBJS     := $(SRC)/msckf_kernels.o $(SRC)/msckf_kalman.o $(SRC)/msckf_gate_mfma.o $(SRC)/msckf_api.o $(SRC)/msckf_frontend.o \
            $(SRC)/msckf_rccl.o
HDRS     := $(SRC)/msckf_common.h $(SRC)/msckf_launch.h $(SRC)/msckf_rchol.h include/msckf_hip.h include/msckf_frontend.h \
            include/msckf_replicas.h

all: $(LIB)

# the gate classes unroll their whole elimination: the pragma-unroll remarks of the
# partial passes before the outer loops are flattened are noise (the ISA is fully unrolled)
$(SRC)/msckf_gate_mfma.o: HIPFLAGS += -Wno-pass-failed

$(SRC)/%.o: $(SRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

# probe build (tools/probes/): same sources with in-kernel phase timers
PROBE    := tools/probes/libmsckf_probe.so
POBJS    := $(patsubst $(SRC)/%.o,tools/probes/obj/%.o,$(OBJS))
probe: $(PROBE)
tools/probes/obj/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p tools/probes/obj
	$(HIPCC) $(HIPFLAGS) -DMSCKF_GATE_PROBE -c $< -o $@
$(PROBE): $(POBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(POBJS) -ldl

clean:
	rm -f $(OBJS) $(LIB) $(PROBE)

.PHONY: all clean probe

# experiment builds (tools/exp_bench.py): the same sources with extra -D flags
#   make exp EXP=kf8 EXPFLAGS=-DMSCKF_IM_KF=8
EXP      ?= exp
EXPFLAGS ?=
EOBJS    := $(patsubst $(SRC)/%.o,tools/exp/obj_$(EXP)/%.o,$(OBJS))
exp: tools/exp/libmsckf_$(EXP).so
tools/exp/obj_$(EXP)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p tools/exp/obj_$(EXP)
	$(HIPCC) $(HIPFLAGS) $(EXPFLAGS) -c $< -o $@
tools/exp/libmsckf_$(EXP).so: $(EOBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(EOBJS) -ldl
.PHONY: exp
