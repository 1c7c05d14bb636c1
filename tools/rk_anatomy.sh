# RANKED backward anatomy (GM_RK_DBG: 0 full, 1 no gathers, 2 no entries), toot 6x4
cd $GRAFT_REPO_ROOT
for cfg in "GM_RK_DBG=0" "GM_RK_DBG=1" "GM_RK_DBG=2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/solve_once.py toot_and_otto_bitstring "length=6,height=4" ranked 3 2>&1 | grep -o '"ms_forward": [0-9.]*, "ms_backward": [0-9.]*'
done
exit 0
