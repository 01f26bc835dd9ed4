#!/bin/bash
# GPU box: the whole-proof VALU ledger (configs[2]): SQ_INSTS_VALU of every prover kernel over 1 and
# over 3 pipelined 64-proof batches (scripts/valu_batches.py), one rocprofv3 --pmc pass each; the
# difference / 128 proofs is the lane-instruction count per proof, by kernel
# (scripts/valu_ledger.py -> gpurun_out/valu/valu_per_proof.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/valu
rm -rf $OUT && mkdir -p $OUT
for B in 1 3; do
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/b$B -o pmc -- python3 scripts/valu_batches.py $B > $OUT/b$B.log 2>&1 || { echo "pass B=$B failed"; tail -5 $OUT/b$B.log; exit 1; }
done
python3 scripts/valu_ledger.py $OUT
# the mix ceiling needs the ISA listings (CPU side, after copying the ledger into profiles/rNN/):
#   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o X.s xfg-stark_amd/csrc/{ntt,kernels,prover}.hip
#   python3 scripts/valu_ceiling.py ntt.s kernels.s prover.s --ledger profiles/rNN/valu_per_proof.json
