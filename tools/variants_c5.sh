# Time the C5 step on library variants (tools/build_variant.sh) and with --fast-math.
set -e
mkdir -p gpurun_out/var
for v in "" ; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --dropin-steps 0 --no-cpu-baseline > gpurun_out/var/c5_default.log 2>&1
  timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --dropin-steps 0 --no-cpu-baseline --fast-math > gpurun_out/var/c5_fast.log 2>&1
done
for v in $VARIANTS; do
  DDR_MC_LIB=ddr_amd/lib/libddr_mc_$v.so timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --dropin-steps 0 --no-cpu-baseline --fast-math > gpurun_out/var/c5_fast_$v.log 2>&1
done
