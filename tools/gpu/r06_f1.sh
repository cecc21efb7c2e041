# final tree: the full GPU suite, smoke, and the headline bench line (default flags)
set -o pipefail
export TAG=${TAG:-f1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 20; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 21; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2>$O/bench.err || { tail -5 $O/bench.err; exit 22; }
tail -1 $O/bench.json | cut -c1-300
