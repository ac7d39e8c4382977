# round 3: (1) training A/B of QAct fc1 at 8 vs 4 waves per workgroup, same box, interleaved;
# (2) k_step PMC records for the current sources (profiles/collect.sh); (3) QAct kernel trace +
# MFMA-busy / HBM counters on the standalone acting forward (profiles/exp_qact.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03n; mkdir -p $O
B="--legs bits --steps 20 --warmup 5 --no-cpu-baseline --eval-mazes 200"
for r in 1 2; do
  timeout -k 10 240 python -u bench.py $B > $O/ab_w8_$r.json 2> $O/ab_w8_$r.err || { tail -20 $O/ab_w8_$r.err; exit 1; }
  MZ_LIB_OVERRIDE=$PWD/profiles/_bin/libmz_q_w4.so timeout -k 10 240 python -u bench.py $B > $O/ab_w4_$r.json 2> $O/ab_w4_$r.err || { tail -20 $O/ab_w4_$r.err; exit 1; }
  python3 -c "import json;[print(t, json.load(open('$O/ab_'+t+'_$r.json'))['win_rate']['train_env_steps_per_s']) for t in ('w8','w4')]"
done
bash profiles/collect.sh || exit 1
echo collect-ok
Q=$O/qact
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $Q/kt -o run -- python3 profiles/exp_qact.py prof > $Q.kt.log 2>&1 || { tail -20 $Q.kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -f csv -d $Q/mfma -o run -- python3 profiles/exp_qact.py prof > $Q.mfma.log 2>&1 || { tail -20 $Q.mfma.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $Q/fetch -o run -- python3 profiles/exp_qact.py prof > $Q.fetch.log 2>&1 || { tail -20 $Q.fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $Q/write -o run -- python3 profiles/exp_qact.py prof > $Q.write.log 2>&1 || { tail -20 $Q.write.log; exit 1; }
echo qact-prof-ok
