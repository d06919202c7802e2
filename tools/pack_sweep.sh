# C5 step time under packer settings, fast-math forward: "COMPFAC QUANT" pairs in $CFGS.
set -e
mkdir -p gpurun_out/pack
for cfg in $CFGS; do
  c=${cfg%,*}; q=${cfg#*,}
  DDR_PACK_COMPFAC=$c DDR_PACK_QUANT=$q timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 \
    --dropin-steps 0 --no-cpu-baseline --fast-math > gpurun_out/pack/c5_cf${c}_q$q.log 2>&1
done
