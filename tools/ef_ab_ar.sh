cd $GRAFT_REPO_ROOT
for ar in 0 0.95; do for v in oldef base; do
  if [ $v = base ]; then L=$PWD/acoss-1_amd/acoss/lib/libacoss_hip.so; else L=$PWD/tools/abl/libabl_$v.so; fi
  echo "== $v ar=$ar"; ACOSS_HIP_LIB=$L timeout -k 10 120 python tools/ef_bench.py --reps 3 --ar $ar 2>&1 | grep -v amdgpu.ids || exit 1
done; done
