export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug_groups.py
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_vs_oracle.py tests/test_gpu_model.py -q -k "fpc_groups or autocast" --timeout 200 --timeout-method thread > gpurun_out/r3e_t.log 2>&1; tail -25 gpurun_out/r3e_t.log
