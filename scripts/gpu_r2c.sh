set -o pipefail
for cfg in "XFG_NTT_E=4" "XFG_NTT_E=5" "XFG_NTT_E=5 XFG_NTT_LTA=8" "XFG_NTT_E=5 XFG_NTT_LTB=9" "XFG_NTT_E=4" "XFG_NTT_E=5"; do
  env $cfg timeout -k 10 120 python3 scripts/lde_shapes.py || exit 1
done
