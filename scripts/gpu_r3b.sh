set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
for v in v_plv v_pls v_nosched v_pls_nosched v_plv; do
  echo "== $v" >> gpurun_out/r3d/micro.txt
  timeout -k 10 120 ./scripts/mb/$v 2>&1 | grep curve >> gpurun_out/r3d/micro.txt || exit 1
done
echo done
