# config-2 trace + per-layer b=1 profile, fp8 parity + config-5 leg (r05)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05o}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_config5_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
tail -n 2 $O/pytest.log
timeout -k 10 200 python3 tools/bench_config5.py > $O/bench_c5.txt 2>&1
tail -n 1 $O/bench_c5.txt | cut -c 1-600
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o t -- python3 tools/trace_config2.py > $O/log.txt 2>&1
python3 tools/trace_config2.py --report $(ls $O/raw/*/t_kernel_trace.csv $O/raw/t_kernel_trace.csv 2>/dev/null | head -n 1) > $O/report.txt
B=1 H=640 W=640 timeout -k 10 200 python3 tools/conv_profile.py > $O/conv_b1.txt 2>&1
timeout -k 10 200 python3 tools/bench_config2.py > $O/bench_c2.txt 2>&1
rm -rf $O/raw
