#!/bin/bash
# checkpoint: hd32 forward occupancy variant + hipBLASLt probe, then the full round measurement
export TMPDIR=/tmp
o=gpurun_out/r3o; mkdir -p $o
VJ_BENCH_ONLY="attn fwd hd32" VJ_BENCH_ROUNDS=9 timeout -k 10 200 python -u tools/bench_kernels.py vjepa2_amd/libvjepa_hip.so vjepa2_amd/libvjepa_hip_f32o5.so > $o/bk.log 2>&1 || { echo "bench failed"; tail -5 $o/bk.log; exit 3; }
cat $o/bk.log
timeout -k 10 200 python -u tools/blaslt_probe.py > $o/blaslt.log 2>&1 || { echo "blaslt probe failed"; tail -5 $o/blaslt.log; exit 6; }
cat $o/blaslt.log
bash tools/gpu_final.sh r03b
