# round 6 (n): why whole h3 train steps differ under CDM_WGRAD_STAGGER=1 (bf16 steps were bit-identical): kernel-level
# slab / sums comparison of the row weight gradient under both schedules, and the h3 train step's run-to-run repeat
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6n
CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out gpurun_out/r6n/k0.npz || exit 1
CDM_WGRAD_STAGGER=1 timeout -k 10 200 python3 tools/wgrad_sched_check.py --out gpurun_out/r6n/k1.npz || exit 1
python3 tools/wgrad_sched_check.py --cmp gpurun_out/r6n/k0.npz gpurun_out/r6n/k1.npz | tee gpurun_out/r6n/kcmp.txt
CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out gpurun_out/r6n/a.npz || exit 1
CDM_WGRAD_STAGGER=0 timeout -k 10 200 python3 tools/tall_check.py --math h3 --out gpurun_out/r6n/b.npz || exit 1
python3 tools/tall_check.py --cmp gpurun_out/r6n/a.npz gpurun_out/r6n/b.npz | tee gpurun_out/r6n/repeat.txt
echo ALL_DONE
