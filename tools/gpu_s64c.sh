cd /root/repo && export TMPDIR=/tmp && o=gpurun_out/s64c && mkdir -p $o
S=vjepa2_amd/libvjepa_hip
for c in "qkv  tgt" "fc2  tgt bf16" "fc1  tgt"; do
  for v in stamps32 stamps; do
    echo "== $v"; VJ_GEMM_STG=1 VJ_STAMPS_LIB=${S}_$v.so timeout -k 10 120 python -u tools/gemm_stamps.py "$c" 2>&1 | grep -v amdgpu.ids || exit 3
  done
done
TAG=s64c STEPS="VJ_LIB=${S}_stg32.so - VJ_GEMM_STG=1" RUNS=2 bash tools/gpu_ab.sh || exit 4
for r in 1 2; do for n in 0 16 32; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/proxy_${n}_$r.log 2>&1 || { echo "proxy $n failed"; tail -5 $o/proxy_${n}_$r.log; exit 5; }
  python3 -c "import json; d=json.loads([l for l in open('$o/proxy_${n}_$r.log') if l.startswith('{')][-1]); print('proxy cus $n run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['allreduce_exposed_ms'], d['dist_backend'])"
done; done
