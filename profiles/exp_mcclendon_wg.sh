set -o pipefail
mkdir -p gpurun_out/r04d
for lib in default profiles/_bin/lib_mc512.so profiles/_bin/lib_mc1024.so default; do
  if [ "$lib" = default ]; then
    timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> gpurun_out/r04d/wg.jsonl || exit 1
  else
    MZ_LIB_OVERRIDE=$lib timeout -k 10 200 python -u profiles/exp_mcclendon_wg.py >> gpurun_out/r04d/wg.jsonl || exit 1
  fi
done
