# A/B of the plane kernel's waves-per-SIMD floor (GM_PLANE_WPE builds of tools/stream_lab), twice each
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  timeout -k 10 100 ./tools/stream_lab 6 0 10 1 || exit 1
  timeout -k 10 100 ./tools/stream_lab_w5 6 0 10 1 || exit 1
done
