set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_gru.py tests/test_gpu_mlp.py tests/test_gpu_decoder_route.py tests/test_autoencoder.py tests/test_gpu_realtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04k.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python3 tools/exp_decoder2.py net net_gemm outmlp outmlp_gemm mlps gru proj dsyn fwd > gpurun_out/dec_r04k.log 2>&1 || exit 1
cat gpurun_out/dec_r04k.log
bash tools/ab_prof.sh gru gru_step gruold grunew gru16h2 gru16h8 || exit 1
cat gpurun_out/ab_prof.log; cp gpurun_out/ab_prof.log gpurun_out/ab_prof_fwd.log
bash tools/ab_prof.sh gru_train gru_bwd_step gruold grunew || exit 1
cat gpurun_out/ab_prof.log
AB_SCRIPT=tools/exp_gru.py bash tools/ab_time.sh gruold grunew || exit 1
cat gpurun_out/ab.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o t -- python3 tools/exp_decoder2.py outmlp outmlp_gemm > gpurun_out/prof_mlp.log 2>&1 || exit 1
echo ALLDONE
