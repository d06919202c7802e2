#!/bin/bash
# Device graph builder: GPU tests, then the C3 training stream with device-built graphs, then C5.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03_dev
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_devgraph.py tests/test_gpu_dropin.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -25 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --stream 10 > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3.json').read()); print('c3', d['ms_per_step'], d['config']['generations_rank0']); print(json.dumps(d['training_stream'])[:900])"
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --dropin-steps 0 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
cut -c1-400 $OUT/c5.json
