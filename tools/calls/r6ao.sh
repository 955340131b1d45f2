# round 6 (ao): final HEAD measurement after the compiled-in B-early halo schedule — full GPU suite, the driver's default bench line, the profiled bench (rocprofv3
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ao
export CDM_PARITY_OUT=$R/gpurun_out/r6ao/parity.jsonl
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6ao/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 gpurun_out/r6ao/tests.log
[ $rc -eq 0 ] || exit 1
unset CDM_PARITY_OUT
timeout -k 10 900 python3 bench.py > gpurun_out/r6ao/bench.json 2> gpurun_out/r6ao/bench.err; echo "bench rc=$?"
python3 -c "import json; b=json.load(open('gpurun_out/r6ao/bench.json')); print('train', b['ms_per_step'], b['value'], b['train_step_stats']['median_ms'], 'sample', b['sample']['ms_per_denoise_step'], b['sample']['img_per_s'], 'cfg', b['sample']['cfg']['w=3']['ms_per_denoise_step'], 'c4', b['configs']['c4_bf16_cfg']['train_ms_per_step'], 'frac', b['roofline']['frac'], 'whole', b['whole_path_roofline']['train_step']['frac'], b['whole_path_roofline']['sample_w=0']['frac'])"
echo ALL_DONE
