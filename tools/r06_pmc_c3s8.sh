# PMC passes on the C3 8-way rank-1 shard alone (light load: VALU per wave-tick of the KR = 1 kernels)
cd $GRAFT_REPO_ROOT
export WORLD_SIZE=8 RANK=1 DDR_BENCH_ALONE=1
bash tools/pmc.sh r06_pmc_c3s8 --workload c3 > gpurun_out/r06_pmc_c3s8.log 2>&1; rc=$?
head -60 gpurun_out/r06_pmc_c3s8/report.txt; exit $rc
