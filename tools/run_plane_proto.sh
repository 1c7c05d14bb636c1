# plane_proto A/B: kernel variant (last argument) 1 = k_plane_resolve_x2, 2 = k_plane_resolve_x2l, 0 = k_plane_resolve
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-v5}
shift
for a in "$@"; do
  timeout -k 5 120 ./tools/plane_proto $a || exit 1
done 2>&1 | tee gpurun_out/plane_proto_$tag.log
