# device gauge union pinned to collate.npz directly
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r06_dev
timeout -k 10 600 python -u -m pytest tests/test_gpu_devgraph.py -v -x --timeout 300 --timeout-method thread > gpurun_out/r06_dev/pytest.log 2>&1; rc=$?
grep -E "passed|failed|Error|assert" gpurun_out/r06_dev/pytest.log | cut -c1-300 | tail -10; exit $rc
