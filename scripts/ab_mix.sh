timeout -k 10 60 ./tools/mix_split_probe > gpurun_out/mixprobe.log 2>&1 && \
timeout -k 10 150 python -u scripts/diag_rollout.py --run --rev HEAD > gpurun_out/diag_ab5.log 2>&1 && \
timeout -k 10 150 python -u scripts/diag_rollout.py --run >> gpurun_out/diag_ab5.log 2>&1 && \
timeout -k 10 200 python -u scripts/diag_fd.py --run --rev HEAD >> gpurun_out/diag_ab5.log 2>&1 && \
timeout -k 10 200 python -u scripts/diag_fd.py --run >> gpurun_out/diag_ab5.log 2>&1 && \
timeout -k 10 200 python -u scripts/diag_fd.py --run --waves 8 >> gpurun_out/diag_ab5.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_update.py tests/test_learn_golden.py tests/test_gpu_rollout_parity.py tests/test_gpu_rollout.py -m gpu -q -x --timeout 120 > gpurun_out/t_mix.log 2>&1; tail -2 gpurun_out/t_mix.log
