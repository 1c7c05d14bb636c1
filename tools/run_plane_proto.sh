set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "4 31 1 5" "5 31 1 5" "4 31 2 5" "5 31 2 3" "6 31 1 20" "6 31 2 10" "6 63 2 5"; do
  timeout -k 5 120 ./tools/plane_proto $a
done 2>&1 | tee gpurun_out/plane_proto_v1.log
