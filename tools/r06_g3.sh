# round 6: GPU suite on the hygiene build, C5 / c3s8 kernel traces vs r05, copy-rate calibration
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_g3
timeout -k 10 120 python tools/copy_bw.py > gpurun_out/r06_g3/copy_bw.txt 2>&1; cat gpurun_out/r06_g3/copy_bw.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_g3/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_g3/pytest.log
[ $rc = 0 ] || exit $rc
LIBS="cur r05" WLS="c5 c3s8" TAG=r06_g3 bash tools/ktrace.sh
