# round 6: GPU suite (cohelp build), then C5 / c3s8 / light kernel traces vs r05
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_g4
timeout -k 10 120 python tools/copy_bw.py > gpurun_out/r06_g4/copy_bw.txt 2>&1; cat gpurun_out/r06_g4/copy_bw.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_g4/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r06_g4/pytest.log
[ $rc = 0 ] || exit $rc
LIBS="cur r05" WLS="c3s8 light c5" TAG=r06_g4 bash tools/ktrace.sh
