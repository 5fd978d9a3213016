cd /root/repo && export TMPDIR=/tmp
S=vjepa2_amd/libvjepa_hip
for c in "qkv  tgt" "fc2  tgt bf16" "fc1  tgt" "qkv  ctx" "dgrad fc2 Wt"; do
  for v in stamps32 stamps; do
    echo "== $v"; VJ_GEMM_STG=1 VJ_STAMPS_LIB=${S}_$v.so timeout -k 10 120 python -u tools/gemm_stamps.py "$c" 2>&1 | grep -v "amdgpu.ids\|spread" || exit 3
  done
done
o=gpurun_out/s64d; mkdir -p $o
for r in 1 2; do for arm in "0 0" "16 0" "16 16" "16 32" "0 16"; do
  set -- $arm; n=$1; res=$2
  VJ_RCCL_RESERVE_CUS=$res timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 --kernel-events 0 --synced-steps 0 --arm-reducer 1 --rccl-proxy-cus $n > $o/proxy_${n}_${res}_$r.log 2>&1 || { echo "proxy $n $res failed"; tail -5 $o/proxy_${n}_${res}_$r.log; exit 5; }
  python3 -c "import json; d=json.loads([l for l in open('$o/proxy_${n}_${res}_$r.log') if l.startswith('{')][-1]); print('proxy cus $n reserve $res run $r', d['value'], d['ms_per_step'], d['ms_per_step_median'], d['allreduce_exposed_ms'], d['dist_backend'])"
done; done
