#!/usr/bin/env python3
"""HBM traffic per launch of k_fixed_accum from two rocprofv3 --pmc passes.

    python3 scripts/pmc_traffic.py TAG RD_STEP WR_STEP WORKLOAD [ROUND]

reads gpurun_out/TAG/pmc_<RD_STEP>/ (TCC_EA0_RDREQ_{32B,64B,128B}_sum) and
gpurun_out/TAG/pmc_<WR_STEP>/ (WRITE_SIZE), the passes `scripts/gpu.sh`'s
`pmc` step runs around `bench.py --serial`, and writes
profiles/<ROUND>_pmc_traffic_<WORKLOAD>.json.

The request-size counters give DRAM bytes directly (every read of this kernel
is a 128-B request: profiles/r02_pmc_fetch_calibration.json), so no FETCH_SIZE
correction applies; WRITE_SIZE is in KiB.  The file carries the SHA-256 of
the measured kernel's machine code as the bench line of the same pass printed
it (roofline.kernel_code), so bench.py attaches it only to lines that ran that
exact kernel, batch and window.
"""
import collections
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(step_dir, prefix):
    """{counter: mean over the k_fixed_accum dispatches} of one pmc pass"""
    paths = glob.glob(os.path.join(step_dir, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit("no counter_collection.csv under %s" % step_dir)
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if prefix not in name.split("(")[0]:
                continue
            # one row per (dispatch, counter); a counter may repeat per agent/XCD: sum them
            vals[r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {c: (sum(d.values()) / len(d), len(d)) for c, d in vals.items()}


def bench_line(step_dir):
    with open(step_dir + ".json") as f:
        for line in f:
            if line.startswith("{"):
                return json.loads(line)
    raise SystemExit("no bench line in %s.json" % step_dir)


def main():
    tag, rd, wr, wl = sys.argv[1:5]
    rnd = sys.argv[5] if len(sys.argv) > 5 else "r04"
    base = os.path.join(ROOT, "gpurun_out", tag)
    line = bench_line(os.path.join(base, "pmc_%s" % rd))
    line_w = bench_line(os.path.join(base, "pmc_%s" % wr))
    kid = line["roofline"]["kernel_code"]
    if kid.get("sha256") != line_w["roofline"]["kernel_code"].get("sha256"):
        raise SystemExit("the two passes ran different kernels")
    curve = line["config"]["curve"]
    prefix = "k_fixed_accum<kzgx::%sG1, %d," % (curve, int(line["config"]["msm"].split("c=")[1].split(",")[0]))
    rdc = per_dispatch(os.path.join(base, "pmc_%s" % rd), prefix)
    wrc = per_dispatch(os.path.join(base, "pmc_%s" % wr), prefix)
    n128 = rdc.get("TCC_EA0_RDREQ_128B_sum", (0, 0))[0]
    n64 = rdc.get("TCC_EA0_RDREQ_64B_sum", (0, 0))[0]
    n32 = rdc.get("TCC_EA0_RDREQ_32B_sum", (0, 0))[0]
    read_b = 128 * n128 + 64 * n64 + 32 * n32
    write_b = wrc["WRITE_SIZE"][0] * 1024
    total = read_b + write_b
    rl = line["roofline"]
    B = line["config"]["batch_per_gpu"]
    fb = int(line["config"]["msm"].split("c=")[1].split(",")[0])
    alg = rl["algorithmic_bytes_per_step"] / rl["launches_per_step"]
    gathered = rl.get("gathered_entry_bytes_per_launch")
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True, text=True).stdout.strip()
    out = {
        "workload": wl,
        "batch": B,
        "fixed_bits": fb,
        "kernel": kid["symbols"][0] if kid.get("symbols") else None,
        "kernel_sha256": kid.get("sha256"),
        "kernel_code_bytes": kid.get("bytes"),
        "git_head": head,
        "source": "rocprofv3 --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum (pass %s), then --pmc WRITE_SIZE (pass %s), "
                  "each on bench.py --serial (gpurun_out/%s, scripts/gpu.sh pmc steps); mean over %d dispatches"
                  % (rd, wr, tag, rdc.get("TCC_EA0_RDREQ_128B_sum", (0, 0))[1]),
        "rdreq_128B_per_launch": n128,
        "rdreq_64B_per_launch": n64,
        "rdreq_32B_per_launch": n32,
        "read_bytes": read_b,
        "write_bytes": write_b,
        "msm_accum_bytes_per_launch": total,
        "algorithmic_bytes_per_launch": alg,
        "gathered_entry_bytes_per_launch": gathered,
        "traffic_over_algorithmic": total / alg,
        "traffic_over_gathered_entries": total / gathered if gathered else None,
        "avg_launch_ms": rl.get("avg_launch_ms"),
        "dram_gbs_during_launch": total / (rl["avg_launch_ms"] * 1e-3) / 1e9 if rl.get("avg_launch_ms") else None,
        "correction": "none: request-size counters are DRAM-side 32/64/128-B request counts",
    }
    path = os.path.join(ROOT, "profiles", "%s_pmc_traffic_%s.json" % (rnd, wl))
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
