# round 6 (o): the early-load staggered weight gradient as the default (CDM_WGRAD_STAGGER=1) with the producer sums'
# contraction pinned — kernel-level and whole-train-step bit-exactness against the lock-step schedule (h3, bf16), then
# the full GPU suite and the driver's default bench line at the new default
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6o; T=/tmp/r6o; mkdir -p $T
CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k0.npz || exit 1
CDM_WGRAD_STAGGER=1 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out $T/k1.npz || exit 1
python3 tools/wgrad_sched_check.py --cmp $T/k0.npz $T/k1.npz | tee gpurun_out/r6o/bitexact.txt
for m in bf16 h3; do
  CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/s0_$m.npz || exit 1
  CDM_WGRAD_STAGGER=1 timeout -k 10 200 python3 tools/tall_check.py --math $m --out $T/s1_$m.npz || exit 1
  python3 tools/tall_check.py --cmp $T/s0_$m.npz $T/s1_$m.npz | sed "s/^/$m train steps: /" | tee -a gpurun_out/r6o/bitexact.txt
done
export CDM_PARITY_OUT=$R/gpurun_out/r6o/parity.jsonl
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r6o/tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/r6o/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python3 bench.py > gpurun_out/r6o/bench.json 2> gpurun_out/r6o/bench.err; echo "bench rc=$?"
python3 -c "import json; b=json.load(open('gpurun_out/r6o/bench.json')); print('train', b['ms_per_step'], b['value'], 'sample', b['sample']['ms_per_denoise_step'], b['sample']['img_per_s'], 'c4', b['configs']['c4_bf16_cfg']['train_ms_per_step'], 'frac', b['roofline']['frac'])"
echo ALL_DONE
