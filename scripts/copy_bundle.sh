#!/bin/bash
# CPU container: copy a final-build bundle (scripts/round_bundle.sh output under gpurun_out/) into
# profiles/$1 (default r06) under the names profiles/*/INDEX.md cites, and add the VALU ledger's
# instruction-mix ceiling from this tree's ISA listings
set -e
R=${1:-r06}
P=profiles/$R
G=gpurun_out
cp $G/round/bench.json $P/bench.json
cp $G/round/summary.json $P/round_summary.json
cp $G/round/trace/bench_kernel_stats.csv $P/bench_kernel_stats.csv
cp $G/round/c5trace/c5_kernel_stats.csv $P/c5_lde_kernel_stats.csv
cp $G/round/lde_pmc.json $P/lde_pmc.json
cp $G/round/lde_pmc_c5.json $P/lde_pmc_c5.json
for i in 1 2 3 4 5; do
  cp $G/round/pmc$i/pmc_counter_collection.csv $P/lde_pmc_pass$i.csv
  cp $G/round/c5pmc$i/pmc_counter_collection.csv $P/lde_pmc_c5_pass$i.csv
done
cp $G/smoke.txt $P/smoke.txt
tail -1 $G/bench_default.json > $P/bench_default.json
cp $G/valu/valu_per_proof.json $P/valu_per_proof.json
cp $G/single_summary.txt $P/single_proof.txt
cp $G/single/single_kernel_stats.csv $P/single_kernel_stats.csv
T=$(mktemp -d /tmp/xfg_isa.XXXX)
for f in ntt kernels prover; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o $T/$f.s xfg-stark_amd/csrc/$f.hip
done
python3 scripts/valu_ceiling.py $T/ntt.s $T/kernels.s $T/prover.s --ledger $P/valu_per_proof.json
rm -rf $T
