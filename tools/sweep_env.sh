cd /root/repo
mkdir -p gpurun_out/sweep
for cfg in "base:" "tgt:VJ_TGT_STREAM=1" "g4:VJ_GEMM_GROUP=4" "g16:VJ_GEMM_GROUP=16" "base2:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --kernel-events 0 > gpurun_out/sweep/$name.log 2>&1 || { echo "$name failed"; exit 3; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/sweep/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'])"
done
