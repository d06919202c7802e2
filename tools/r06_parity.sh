# element-wise gradient bars: fp64 kernel vs fp64 oracle, exact adjoint vs the fp64 adjoint of the same trajectory
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r06_parity
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact_adjoint.py tests/test_gpu_route.py -v -s -x --timeout 300 --timeout-method thread \
  > gpurun_out/r06_parity/pytest.log 2>&1; rc=$?
grep -E "passed|failed|normrel|Error|assert" gpurun_out/r06_parity/pytest.log | cut -c1-400 | tail -30; exit $rc
