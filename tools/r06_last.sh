# last check on the final tree: full -m gpu suite, smoke, the default bench line
cd $GRAFT_REPO_ROOT; O=gpurun_out/r06_last; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | cut -c1-300
