cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_g1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_g1/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r06_g1/pytest.log
[ $rc = 0 ] || exit $rc
LIBS="cur r05" WLS="c5 c3s8" TAG=r06_g1 bash tools/ktrace.sh
