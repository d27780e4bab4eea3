cd $GRAFT_REPO_ROOT
for d in 0 1 2; do for tile in -1 0 1; do
  e="DDIM_COLD_GEMM_DEBUG=$d"; [ $tile -ge 0 ] && e="$e DDIM_COLD_GEMM_TILE=$tile"
  env $e timeout -k 5 120 python tools/ub_sampler_ends.py 2>/dev/null || exit 1
done; done
