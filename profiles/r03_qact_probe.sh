set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_qact.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u profiles/exp_qact.py main > $O/probe.jsonl || exit 1
for v in w8; do
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/libmz_q_$v.so timeout -k 10 120 python -u profiles/exp_qact.py $v >> $O/probe.jsonl || exit 1
done
MZ_LIB_OVERRIDE=$PWD/profiles/_bin/libmz_q_w8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_qact.py > $O/tests_il6.log 2>&1 || { tail -30 $O/tests_il6.log; exit 1; }
tail -1 $O/tests_il6.log
cat $O/probe.jsonl
