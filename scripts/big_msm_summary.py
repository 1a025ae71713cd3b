"""Summarise a scripts/big_msm.py run under rocprofv3 (gpu.sh profpy step):
per size, the median time of the whole MSM and of every kernel it launched
(kernel trace), plus any pmcpy counter passes of the accumulation kernels.

    python3 scripts/big_msm_summary.py gpurun_out/TAG OUT.json"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, out):
    rec = {"source": d, "sizes": []}
    for txt in sorted(glob.glob(os.path.join(d, "profpy_*.txt"))):
        runs = [json.loads(l) for l in open(txt) if l.startswith("{") and "srs_points" in l]
        trace = os.path.join(txt[:-4], "prof_kernel_trace.csv")
        if not runs or not os.path.exists(trace):
            continue
        rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
        msm, per = -1, collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            n = r["Kernel_Name"]
            if "k_big2_count" in n or "k_big_count" in n:
                msm += 1
            if msm < 0 or any(x in n for x in ("gen_srs", "table_build", "at::", "srs_to", "copyBuffer")):
                continue
            short = n.split("(")[0].replace("void ", "").replace("kzgx::", "")
            per[msm // 9][short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for s, run in enumerate(runs):
            ks = {k: sorted(v)[len(v) // 2] for k, v in per[s].items()}
            rec["sizes"].append({**run, "kernel_us_median": ks})
    pmc = {}
    for f in sorted(glob.glob(os.path.join(d, "pmcpy_*", "pmc_counter_collection.csv"))):
        agg, cnt = collections.defaultdict(float), collections.Counter()
        for r in csv.DictReader(open(f)):
            if "accum" in r["Kernel_Name"]:
                k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Counter_Name"])
                agg[k] += float(r["Counter_Value"])
                cnt[k] += 1
        pmc[f] = {f"{k[0]} {k[1]}": v / cnt[k] for k, v in sorted(agg.items())}
    rec["pmc_per_launch"] = pmc
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec)[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
