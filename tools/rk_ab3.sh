# RANKED block-order A/B (GM_RK_ORDER), toot 6x4, each twice
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for cfg in "GM_RK_ORDER=code" "GM_RK_ORDER=morton"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 3 2>&1 | grep -o '"ms_forward": [0-9.]*, "ms_backward": [0-9.]*\|"root_line": "[^"]*"' || exit 1
done; done
