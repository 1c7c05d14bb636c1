cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "2 31 1 2 1" "3 3 1 2 1" "4 31 1 5 1" "4 31 2 5 1" "5 31 1 3 1" "5 31 2 3 1" "6 31 1 20 1" "6 31 1 20 0" "6 31 2 10 1" "6 31 2 10 0" "6 63 2 5 1"; do
  timeout -k 5 120 ./tools/plane_proto $a
done 2>&1 | tee gpurun_out/plane_proto_v4.log
