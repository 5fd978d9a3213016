mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -s tests/test_gpu_kernels.py tests/test_gpu_model.py -k "epilogues or jepa_loss or target_bf16 or train_steps or checkpoint_resume" > gpurun_out/bt.log 2>&1 || { echo tests failed; tail -30 gpurun_out/bt.log; exit 1; }
grep -E "passed|failed|mean\|" gpurun_out/bt.log | tail -5
for i in 1 2; do for v in 1 0; do VJ_TARGET_BF16=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --cpu-baseline 0 --kernel-events 0 > gpurun_out/bb_$v.$i.log 2>&1 || { echo bench failed; tail gpurun_out/bb_$v.$i.log; exit 1; }; python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/bb_$v.$i.log') if l.startswith('{')][-1]); print('bf16=$v', d['value'], d['ms_per_step'], d['loss_last'])"; done; done
