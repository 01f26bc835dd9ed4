"""Summaries of a scripts/profile_round.sh bundle: kernel stats of the bench command, the trace-LDE
launch durations inside it (the xfg_bench_lde launch sets bench.py times with HIP events), and the
PMC of the trace-LDE launch sets alone for configs[2] (pmc*/) and configs[4] (c5pmc*/): traffic =
FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md HBM section; rocprofv3 reports both in KB), VALU
instructions and stall split per pass. Writes summary.json, lde_pmc.json and lde_pmc_c5.json (the
records bench.py reads for its `traffic` fields) into the bundle directory."""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1]


def rows(pattern):
    f = glob.glob(os.path.join(out, pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def kind(name):
    return "a" if "ntt_pass_a" in name else ("b" if "ntt_pass_b" in name else None)


bench = json.loads(open(os.path.join(out, "bench.json")).read().strip().splitlines()[-1])
res = {"bench_value": bench["value"], "bench_ms_per_step": bench["ms_per_step"], "bench_roofline": bench["roofline"],
       "bench_whole_proof": bench.get("whole_proof"), "bench_config5": bench.get("config5")}

# the last trace-LDE launch sets of the bench trace: pass A / B kernels with the 64-proof grid
tr = rows("trace/**/*kernel_trace.csv")
grid = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], grid(r)) for r in tr)
big = defaultdict(int)
for e in ev:
    if kind(e[2]):
        big[(kind(e[2]), e[2], e[3])] += 1
# the grids of the 64-proof (448-column) trace LDE are the largest pass-A / pass-B grids at 2^16 x 8
sel = {}
for k in ("a", "b"):
    cand = [(g, nm) for (kk, nm, g) in big if kk == k and "cos" in nm] if k == "a" else \
           [(g, nm) for (kk, nm, g) in big if kk == k and ("<8, false, 8, 4>" in nm or "ntt_pass_b_tq" in nm)]
    if cand:
        sel[k] = max(cand)
if len(sel) == 2:
    a = [e for e in ev if (e[3], e[2]) == sel["a"]]
    b = [e for e in ev if (e[3], e[2]) == sel["b"]]
    k = min(10, len(a), len(b))
    if k:
        da = sum(e[1] - e[0] for e in a[-k:]) / k / 1e6
        db = sum(e[1] - e[0] for e in b[-k:]) / k / 1e6
        res["rocprof_lde_launch_set"] = {"pass_a": sel["a"][1], "pass_b": sel["b"][1], "pass_a_ms": round(da, 4),
                                         "pass_b_ms": round(db, 4), "sum_ms": round(da + db, 4), "launch_sets": k}

mean = lambda v: sum(v) / len(v) if v else 0.0


def pmc(prefix, count, n, blowup):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, prefix + "*/**/*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if "a" not in acc or "b" not in acc:
        return None
    fetch = 2 * 1024 * (mean(acc["a"]["FETCH_SIZE"]) + mean(acc["b"]["FETCH_SIZE"]))
    write = 1024 * (mean(acc["a"]["WRITE_SIZE"]) + mean(acc["b"]["WRITE_SIZE"]))
    outputs = 7 * count * n * blowup
    d = {"count": count, "n": n, "blowup": blowup, "traffic_bytes": int(fetch + write), "fetch_bytes_x2": int(fetch),
         "write_bytes": int(write), "algorithmic_bytes": 8 * 7 * (n + n * blowup) * count}
    for k in ("a", "b"):
        c = acc[k]
        d[f"valu_insts_pass_{k}"] = mean(c.get("SQ_INSTS_VALU", []))
        d[f"lane_instr_per_output_pass_{k}"] = round(64 * mean(c.get("SQ_INSTS_VALU", [])) / outputs, 1)
        d[f"valu_busy_pct_pass_{k}"] = round(mean(c.get("VALUBusy", [])), 1)
        d[f"occupancy_pct_pass_{k}"] = round(mean(c.get("OccupancyPercent", [])), 1)
        wc = mean(c.get("SQ_WAVE_CYCLES", []))
        if wc:
            d[f"stall_split_pass_{k}"] = {s: round(mean(c.get(s, [])) / wc, 3)
                                          for s in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")}
    d["traffic_over_algorithmic"] = round(d["traffic_bytes"] / d["algorithmic_bytes"], 3)
    return d


for prefix, name, shape in (("pmc", "lde_pmc.json", (64, 65536, 8)), ("c5pmc", "lde_pmc_c5.json", (4, 1 << 20, 16))):
    d = pmc(prefix, *shape)
    if d:
        res[name] = d
        json.dump(d, open(os.path.join(out, name), "w"), indent=1)

stats = rows("trace/**/*kernel_stats.csv")
res["top_kernels"] = [{"name": r["Name"][:80], "calls": int(r["Calls"]), "total_ms": round(float(r["TotalDurationNs"]) / 1e6, 3),
                       "avg_us": round(float(r["AverageNs"]) / 1e3, 2)} for r in stats[:15]]
c5 = rows("c5trace/**/*kernel_stats.csv")
res["c5_lde_kernels"] = [{"name": r["Name"][:80], "calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
                         for r in c5[:4]]
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "top_kernels"}, indent=1))
