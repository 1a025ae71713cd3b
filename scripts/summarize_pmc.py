#!/usr/bin/env python3
"""Summarize rocprofv3 PMC passes (gpurun_out/pmc/<COUNTER>/run_counter_collection.csv)
into profiles/: per-kernel mean counters, and the accum kernel's HBM traffic per
launch for bench.py's roofline.traffic (FETCH_SIZE x2 per MI355X_MICROARCH.md)."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
out = {}
for t in sorted(os.listdir(os.path.join(ROOT, "gpurun_out", "pmc"))):
    path = os.path.join(ROOT, "gpurun_out", "pmc", t, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        for c, x in v.items():
            out.setdefault(k, {})[c] = {"dispatches": len(x), "mean_per_dispatch": sum(x) / len(x)}
json.dump(out, open(os.path.join(ROOT, "profiles", "%s_pmc_counters_cfg2.json" % tag), "w"), indent=1)
acc = next(v for k, v in out.items() if k.startswith("kzgx::k_fixed_accum<kzgx::BN254G1"))
fetch_raw = acc["FETCH_SIZE"]["mean_per_dispatch"] * 1024
write = acc["WRITE_SIZE"]["mean_per_dispatch"] * 1024
tr = {
    "workload": "cfg2", "batch": batch, "kernel": "k_fixed_accum<BN254G1,16>",
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on bench.py --serial --steps 2 "
              "--warmup 1; scripts/summarize_pmc.py",
    "fetch_size_raw_bytes": fetch_raw,
    "fetch_bytes_corrected": 2 * fetch_raw,
    "write_bytes": write,
    "msm_accum_bytes_per_launch": 2 * fetch_raw + write,
    "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: gfx950 tallies 128-B requests at 64 B for "
                  "16-B/lane loads; the table gathers are 5 x dwordx4 per lane per term)",
    "table_bytes_read_algorithmic": batch * 4097 * 16 * 80,
}
json.dump(tr, open(os.path.join(ROOT, "profiles", "pmc_traffic_cfg2.json"), "w"), indent=1)
print(json.dumps(tr, indent=1))
