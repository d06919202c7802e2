cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r06_ew
timeout -k 10 600 python -u -m pytest tests/test_gpu_route.py -v -x -k "elementwise" --timeout 300 --timeout-method thread > gpurun_out/r06_ew/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert|PASS|FAIL" gpurun_out/r06_ew/pytest.log | cut -c1-300 | tail -12; exit $rc
