"""Summarise scripts/valu_ledger.sh: per kernel name, SQ_INSTS_VALU summed over all dispatches in the
B = 3 run minus the B = 1 run, x 64 lanes / 128 proofs = lane instructions per proof; writes
valu_per_proof.json (the record bench.py's whole_proof.valu reads from profiles/rNN/)."""
import collections
import csv
import glob
import json
import os
import sys

out = sys.argv[1]


def totals(d):
    acc = collections.defaultdict(float)
    for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "SQ_INSTS_VALU":
                acc[r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"])
    return acc


t1, t3 = totals("b1"), totals("b3")
proofs = 128
per = {k: 64.0 * (t3[k] - t1.get(k, 0.0)) / proofs for k in t3}
per = {k: v for k, v in per.items() if v > 0}
tot = sum(per.values())
rec = {"workload": "configs[2]: 64-proof batches, n = 2^16, beta 8, 42/8/4/None/8/31",
       "method": "rocprofv3 --pmc SQ_INSTS_VALU over 3 and over 1 pipelined batches, difference x 64 lanes / 128 proofs",
       "lane_instr_per_proof": round(tot), "by_kernel": {k: round(v) for k, v in sorted(per.items(), key=lambda x: -x[1])}}
rec["share"] = {k: round(v / tot, 4) for k, v in sorted(per.items(), key=lambda x: -x[1])[:12]}
json.dump(rec, open(os.path.join(out, "valu_per_proof.json"), "w"), indent=1)
print(json.dumps(rec, indent=1))
