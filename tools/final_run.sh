set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --tune-save gpurun_out/tune_final.json > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
TAG=final TUNE=gpurun_out/tune_final.json CONV_TIMING=both timeout -k 10 400 bash tools/gpu_profile.sh > gpurun_out/final_prof.log 2>&1
TAG=pmc_final timeout -k 10 600 bash tools/gpu_pmc.sh > gpurun_out/pmc_final.log 2>&1
