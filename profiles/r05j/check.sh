#!/bin/bash
# round 5: (1) where k_mcclendon's time goes now (MZ_MC_PROBE: return after phase k); (2) the
# bits-mode k_step floor (MZ_PROBE 128: return at once; 256: no level-2 gathers) and its batch
# sweep; (3) the K-update graph in the live trainer (round-4 package twice, current twice,
# MZ_K_BLOCK=1); (4) training traces (DDQN headline leg, config 4) -> per-stream breakdown
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export PYTHONUNBUFFERED=1
R=$(pwd)
for lib in default 5 6 7; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_mcp$lib.so; fi
  timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> $O/mc_probes.jsonl || exit 1
done
for lib in default probe128 probe256 default; do
  if [ $lib = default ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=profiles/_bin/lib_$lib.so; fi
  timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 --legs bits --train-steps 0 --curriculum-steps 0 \
    --config-legs "" --no-cpu-baseline > $O/bits_$lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/bits_$lib.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'$lib','envs':65536,'value':d['value'],'ms':d['ms_per_step'],'kernel_ms':d['roofline']['avg_kernel_ms']}))" >> $O/bits_floor.jsonl
done
unset MZ_LIB_OVERRIDE
for envs in 16384 32768 131072 262144; do
  timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 --legs bits --envs $envs --train-steps 0 --curriculum-steps 0 \
    --config-legs "" --no-cpu-baseline > $O/bits_$envs.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('$O/bits_$envs.json').read().strip().splitlines()[-1]);print(json.dumps({'lib':'default','envs':$envs,'value':d['value'],'ms':d['ms_per_step'],'kernel_ms':d['roofline']['avg_kernel_ms']}))" >> $O/bits_floor.jsonl
done
for pkg in old old new new; do
  MZ_K_BLOCK=1 timeout -k 10 400 python -u profiles/r05f/kblock_repro.py $pkg >> $O/kblock.jsonl 2>> $O/kblock.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr/kt -o run -- python3 bench.py --steps 10 --warmup 2 --train-steps 300 --no-cpu-baseline --eval-mazes 64 --curriculum-steps 0 --config-legs= > $O/kt.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr/kt/run_kernel_trace.csv --skip 50 --top 25 > $O/train_streams.json || exit 1
cp /tmp/tr/kt/run_kernel_stats.csv $O/train_kernel_stats.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/tr4/kt -o run -- python3 bench.py --legs bits --steps 10 --warmup 2 --train-steps 0 --curriculum-steps 0 --no-cpu-baseline --config-legs cfg4 --cfg4-steps 300 --cfg-eval-mazes 32 > $O/kt4.log 2>&1 || exit 1
python3 profiles/train_streams.py /tmp/tr4/kt/run_kernel_trace.csv --skip 50 --top 25 --step-kernel "k_step<4, false, true, true, false>" > $O/cfg4_train_streams.json || exit 1
cp /tmp/tr4/kt/run_kernel_stats.csv $O/cfg4_kernel_stats.csv
