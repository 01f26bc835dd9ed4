"""Summaries of a scripts/profile_round.sh bundle: kernel stats of the bench command, the trace-LDE
launch durations inside it (the xfg_bench_lde launch sets bench.py times with HIP events), and the
PMC traffic of those launch sets (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section;
rocprofv3 reports both in KB)."""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1]
PA, PB = "void xfg::ntt_pass_a_cos<8>(xfg::NttArgs)", "void xfg::ntt_pass_b<8, false, 8, 4>(xfg::NttArgs)"
# grids (threads) of the trace-LDE launch set, 7 columns x 64 proofs at n = 2^16: pass A one block per
# (16-column tile, column) covering all 8 cosets, pass B one thread per 16 outputs
GRID = {PA: 16 * 448 * 256, PB: 14680064}

def rows(pattern):
    f = glob.glob(os.path.join(out, pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []

bench = json.loads(open(os.path.join(out, "bench.json")).read().strip().splitlines()[-1])
res = {"bench_value": bench["value"], "bench_ms_per_step": bench["ms_per_step"], "bench_roofline": bench["roofline"]}
# the last launch sets of pass A/B with the trace-LDE grid are xfg_bench_lde's timed launches
tr = rows("trace/**/*kernel_trace.csv")
grid = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid(r)) for r in tr)
a = [e for e in ev if e[2] == PA and e[3] == GRID[PA]]
b = [e for e in ev if e[2] == PB and e[3] == GRID[PB]]
k = min(10, len(a), len(b))
if k:
    da = sum(e[1] - e[0] for e in a[-k:]) / k / 1e6
    db = sum(e[1] - e[0] for e in b[-k:]) / k / 1e6
    res["rocprof_lde_launch_set"] = {"pass_a_ms": round(da, 4), "pass_b_ms": round(db, 4), "sum_ms": round(da + db, 4),
                                     "launch_sets": k, "bench_hip_event_ms": float(bench["roofline"]["kernel"].split(" ms/launch-set")[0].split(", ")[-1])}
# PMC
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "pmc*/**/*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if GRID.get(r["Kernel_Name"]) == int(r["Grid_Size"]):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = lambda v: sum(v) / len(v) if v else 0.0
if PA in acc and PB in acc:
    fetch = 2 * 1024 * (mean(acc[PA]["FETCH_SIZE"]) + mean(acc[PB]["FETCH_SIZE"]))
    write = 1024 * (mean(acc[PA]["WRITE_SIZE"]) + mean(acc[PB]["WRITE_SIZE"]))
    res["lde_pmc"] = {"count": 64, "n": 65536, "blowup": 8, "traffic_bytes": int(fetch + write),
                      "fetch_bytes_x2": int(fetch), "write_bytes": int(write),
                      "valu_insts_pass_a": mean(acc[PA].get("SQ_INSTS_VALU", [])),
                      "valu_insts_pass_b": mean(acc[PB].get("SQ_INSTS_VALU", [])),
                      "valu_busy_pct_pass_a": round(mean(acc[PA].get("VALUBusy", [])), 1),
                      "valu_busy_pct_pass_b": round(mean(acc[PB].get("VALUBusy", [])), 1),
                      "occupancy_pct_pass_a": round(mean(acc[PA].get("OccupancyPercent", [])), 1),
                      "occupancy_pct_pass_b": round(mean(acc[PB].get("OccupancyPercent", [])), 1),
                      "algorithmic_bytes": 8 * 7 * (65536 + 8 * 65536) * 64}
stats = rows("trace/**/*kernel_stats.csv")
res["top_kernels"] = [{"name": r["Name"][:80], "calls": int(r["Calls"]), "total_ms": round(float(r["TotalDurationNs"]) / 1e6, 3),
                       "avg_us": round(float(r["AverageNs"]) / 1e3, 2)} for r in stats[:15]]
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "top_kernels"}, indent=1))
