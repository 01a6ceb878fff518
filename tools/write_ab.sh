#!/bin/bash
# WRITE_SIZE / FETCH_SIZE and kernel time of one acoss_crp_align call (kbench, one stream) for the
# in-tree library and a tools/abl variant:  bash tools/write_ab.sh VARIANT [frames]
set -euo pipefail
V=$1; F=${2:-2000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/write_ab
mkdir -p "$OUT"
export TMPDIR=/tmp ACOSS_SPLIT_STREAMS=1
cd /tmp
for v in base "$V"; do
  if [ "$v" = base ]; then L=$R/acoss-1_amd/acoss/lib/libacoss_hip.so; else L=$R/tools/abl/libabl_$v.so; fi
  B="$R/tools/kbench.py --frames $F --pairs 13366 --reps 1 --noprof"
  ACOSS_HIP_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/$v/w" -o run -- python3 $B > "$OUT/$v.w.log" 2>&1
  ACOSS_HIP_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$v/kt" -o run -- python3 $B > "$OUT/$v.kt.log" 2>&1
done
echo done
