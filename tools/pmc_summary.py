"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_summary.json.

    python tools/pmc_summary.py FETCH.csv WRITE.csv --steps K --dtype fp32 [-o profiles/pmc_summary.json]

FETCH.csv / WRITE.csv are the counter_collection CSVs of two separate
`rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs of the same
`bench.py --steps K --warmup 0` command (the two TCC counters do not fit in
one pass on gfx950).  Counter values are KiB per dispatch.  Kernels are
grouped into the bench's timer stages; bytes_per_step = (FETCH + WRITE) * 1024
per dispatch, summed over the stage's kernels (each runs once per step).  Per MI355X_MICROARCH.md, FETCH_SIZE on
gfx950 reads half of a 16-B-per-lane streaming read and other access widths
are uncalibrated, so `fetch_x2_bytes_per_step` gives the upper estimate.
"""
import argparse
import csv
import json
import re
from collections import defaultdict

STAGES = [
    ("triangulate", r"k_triangulate"),
    ("feature_jacobian", r"k_feature"),
    ("gate", r"k_gate"),
    ("select", r"k_select"),
    ("compress", r"k_info|k_compress|k_widen"),
    ("kalman_a", r"k_kal_a|k_kal_mchol<\w+, \d+, \d+, 0|k_gchol_a_|k_gchol_\w+<0"),
    ("kalman_b", r"k_kal_b"),
    ("kalman_c", r"k_kal_c|k_kal_mchol<\w+, \d+, \d+, 1|k_gchol_c_|k_gchol_\w+<1"),
    ("kalman_e", r"k_kal_e"),
    ("kalman_correct", r"k_correct"),
]


def stage_of(name):
    for st, pat in STAGES:
        if re.search(pat, name):
            return st
    return None


def short_name(name):
    """Kernel name without its return type, namespaces and argument list:
    'void msckf::(anonymous namespace)::k_gate_mfma<float, 6, true>(msckf::...)'
    -> 'k_gate_mfma<float, 6, true>'.  The argument list is the LAST top-level
    parenthesis group (the '(anonymous namespace)' qualifier also has one, so
    cutting at the first '(' would collapse every anonymous-namespace kernel
    to one key)."""
    n = name.strip()
    depth, cut = 0, len(n)
    for i in range(len(n) - 1, -1, -1):
        c = n[i]
        if c == ")":
            depth += 1
        elif c == "(":
            depth -= 1
            if depth == 0:
                cut = i
                break
    n = n[:cut] if cut < len(n) and n.endswith(")") else n
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.replace("msckf::", "")


def read(path):
    out = defaultdict(float)
    count = defaultdict(int)
    for row in csv.DictReader(open(path)):
        name = row["Kernel_Name"]
        out[name] += float(row["Counter_Value"])
        count[name] += 1
    return out, count


def workload_of_log(path):
    """(workload key, dtype) of the bench line in a bench.py log (the last JSON line)."""
    line = None
    for ln in open(path):
        ln = ln.strip()
        if ln.startswith("{") and '"config"' in ln:
            line = ln
    if line is None:
        return None, None
    d = json.loads(line)
    c = d["config"]
    return ("N%dxF%dxB%d" % (c["cam_states"], c["features"], c["filters_per_gpu"]),
            "fp64" if d.get("dtype") == "f64" else "fp32")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--steps", type=int, default=0,
                    help="update steps in the passes (default: the dispatches of k_select of --dtype, one per step)")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("-o", "--out", default="profiles/pmc_summary.json")
    ap.add_argument("--source", default="")
    ap.add_argument("--workload", default=None,
                    help="bench workload the passes ran, N<cams>xF<features>xB<filters> (bench.py only uses the "
                         "traffic for the same one); default: read from --bench-log, else N30xF200xB2048")
    ap.add_argument("--bench-log", default=None,
                    help="log of the pass's bench.py run: its JSON line gives the workload (and --dtype)")
    a = ap.parse_args()
    if a.bench_log:
        wl, dt = workload_of_log(a.bench_log)
        a.workload = a.workload or wl
        a.dtype = dt or a.dtype
    a.workload = a.workload or "N30xF200xB2048"
    fetch, nf = read(a.fetch)
    write, nw = read(a.write)
    tname = "float" if a.dtype == "fp32" else "double"
    if a.steps <= 0:   # every update runs k_select exactly once
        a.steps = sum(c for n, c in nf.items() if "k_select<%s" % tname in n)
        assert a.steps > 0, "no k_select dispatch of %s in %s" % (tname, a.fetch)
    stages = {}
    for name in sorted(set(fetch) | set(write)):
        if "<%s" % ("double" if tname == "float" else "float") in name:
            continue   # the other context's kernels (bench legs of the other scalar type)
        st = stage_of(name)
        if st is None:
            continue
        d = stages.setdefault(st, {"fetch_kib": 0.0, "write_kib": 0.0, "kernels": {}})
        d["fetch_kib"] += fetch.get(name, 0.0)
        d["write_kib"] += write.get(name, 0.0)
        short = short_name(name)
        assert short not in d["kernels"], "kernel key collision: %s" % short
        d["kernels"][short] = {"dispatches": nf.get(name, nw.get(name, 0)),
                               "fetch_kib": fetch.get(name, 0.0), "write_kib": write.get(name, 0.0)}
    # every kernel of a stage runs once per update step: per-dispatch averages
    # (the bench's no-triangulation leg skips k_triangulate, so dispatch counts differ)
    for st, d in stages.items():
        f = sum(k["fetch_kib"] / max(k["dispatches"], 1) for k in d["kernels"].values())
        w = sum(k["write_kib"] / max(k["dispatches"], 1) for k in d["kernels"].values())
        d["bytes_per_step"] = (f + w) * 1024
        d["fetch_x2_bytes_per_step"] = (2 * f + w) * 1024
    json.dump({"dtype": a.dtype, "steps": a.steps, "workload": a.workload, "source": a.source, "unit": "bytes",
               "stages": stages}, open(a.out, "w"), indent=1, sort_keys=True)
    for st, d in sorted(stages.items(), key=lambda kv: -kv[1]["bytes_per_step"]):
        print("%-18s %10.3f GB/step" % (st, d["bytes_per_step"] / 1e9))


if __name__ == "__main__":
    main()
