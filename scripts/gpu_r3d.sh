#!/bin/bash
# per-regime VALU of the wave-staged kernel (variant 209: <= 3 objects/wave, all staged)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/rc209; mkdir -p $O
bash scripts/regime_costs.sh rc 209 "u8 u24 u48 u100 u150 num flt cfg3b" > $O/regime_costs_v209.txt 2>&1 || { tail $O/regime_costs_v209.txt; exit 1; }
cat $O/regime_costs_v209.txt
