cd $GRAFT_REPO_ROOT
for t in default 0 1 2; do
  if [ $t = default ]; then timeout -k 10 120 python tools/ub_gemm_phase.py || exit 1
  else DDIM_COLD_GEMM_TILE=$t timeout -k 10 120 python tools/ub_gemm_phase.py || exit 1; fi
done
