"""copy the judged pieces of a scripts/profile_round.sh bundle (gpurun_out/round) into profiles/<tag>/"""
import glob, json, os, shutil, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "gpurun_out", "round")
dst = os.path.join(ROOT, "profiles", sys.argv[1] if len(sys.argv) > 1 else "r01")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))
shutil.copy(glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)[0],
            os.path.join(dst, "bench_kernel_stats.csv"))
summ = json.load(open(os.path.join(src, "summary.json")))
json.dump(summ, open(os.path.join(dst, "round_summary.json"), "w"), indent=1)
json.dump(summ["lde_pmc"], open(os.path.join(dst, "lde_pmc.json"), "w"), indent=1)
for f in glob.glob(os.path.join(dst, "lde_pmc_pass*.csv")):
    os.remove(f)
for i, f in enumerate(sorted(glob.glob(os.path.join(src, "pmc*", "**", "*counter_collection.csv"), recursive=True)), 1):
    shutil.copy(f, os.path.join(dst, f"lde_pmc_pass{i}.csv"))
print("profiles ->", os.path.relpath(dst, ROOT), sorted(os.listdir(dst)))
