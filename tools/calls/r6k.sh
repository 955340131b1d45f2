# round 6 (k): HEAD measurement — the driver's default bench line (N=1, every leg), then rocprofv3 kernel trace + stats
# of the short bench with the CFG legs on and the PMC passes on the dominant conv (tools/gpu_profile.sh), then the PMC
# families of the C2 train step (tools/pmc_step.sh)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6k
timeout -k 10 900 python3 bench.py > gpurun_out/r6k/bench.json 2> gpurun_out/r6k/bench.err; echo "bench rc=$?"
python3 -c "import json; b=json.load(open('gpurun_out/r6k/bench.json')); print('train', b['ms_per_step'], b['value'], 'sample', b['sample']['ms_per_denoise_step'], b['sample']['img_per_s'], 'c4', b['configs']['c4_bf16_cfg']['train_ms_per_step'], 'frac', b['roofline']['frac'])"
timeout -k 10 1000 bash tools/gpu_profile.sh gpurun_out/r6k h3; echo "prof rc=$?"
python3 tools/kstats.py gpurun_out/r6k/trace/bench_kernel_stats.csv > gpurun_out/r6k/summary.txt && head -8 gpurun_out/r6k/summary.txt
timeout -k 10 600 bash tools/pmc_step.sh gpurun_out/r6k/pmc_step > gpurun_out/r6k/pmc_step.txt 2>&1; echo "pmc step rc=$?"
echo ALL_DONE
