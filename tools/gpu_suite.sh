cd /root/repo && export TMPDIR=/tmp
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('bench', d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline']['value'])
for l in d['legs']: print(l['leg'], l['value'], l['roofline']['kernel'], l['roofline']['frac'])"
