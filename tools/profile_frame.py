"""Where the drop-in per-frame path's time goes: replays the golden synthetic
stream s1 through msckf_amd.MSCKF (fp64, one filter) and reports frames/s,
the wall time per device request kind (each served by one C-ABI call), and
the top host functions under cProfile.

    python tools/profile_frame.py [--frames 200] [--cprofile]
"""
import argparse
import cProfile
import json
import os
import pstats
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import msckf_pkg  # noqa: E402,F401
import msckf_amd  # noqa: E402
from msckf_amd import synth  # noqa: E402
from msckf_amd.replay import FeatureStream, replay  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cprofile", action="store_true")
    a = ap.parse_args()
    st = FeatureStream.from_synthetic(synth.make_sequence(a.frames, a.seed))
    flt = msckf_amd.MSCKF()
    replay(flt, FeatureStream.from_synthetic(synth.make_sequence(30, a.seed)))   # warm-up (kernels loaded)
    flt.close()
    flt = msckf_amd.MSCKF()
    tot, cnt = defaultdict(float), defaultdict(int)
    serve = flt._serve

    def timed(req):
        t0 = time.perf_counter()
        r = serve(req)
        tot[req[0]] += time.perf_counter() - t0
        cnt[req[0]] += 1
        return r
    flt._serve = timed
    prof = cProfile.Profile() if a.cprofile else None
    ev = st.events()   # the front-end's messages, outside the timed region
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    traj = replay(flt, st, events=ev)
    if prof:
        prof.disable()
    el = time.perf_counter() - t0
    flt.close()
    n = len(traj)
    out = {"frames": n, "frames_per_s": round(n / el, 1), "ms_per_frame": round(el / n * 1e3, 3),
           "device_requests_ms_per_frame": {k: round(v / n * 1e3, 4) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])},
           "requests_per_frame": {k: round(v / n, 2) for k, v in cnt.items()},
           "host_ms_per_frame": round((el - sum(tot.values())) / n * 1e3, 3)}
    print(json.dumps(out), flush=True)
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
