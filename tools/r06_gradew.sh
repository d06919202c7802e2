cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r06_gradew
timeout -k 10 300 python tools/dbg/grad_elementwise.py > gpurun_out/r06_gradew/out.txt 2>&1; rc=$?; cat gpurun_out/r06_gradew/out.txt | grep -v amdgpu.ids; exit $rc
