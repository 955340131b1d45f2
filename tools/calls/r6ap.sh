# round 6 (ap): the three-barrier halo schedule's last-row stores without the `more chunks` condition (they store the
# next tile's chunk 0 in place of the post-loop stores) — kernel tests + whole-step bit-exactness (h3) against HEAD's
# build, then same-box A/B (sampling, C2)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ap; T=/tmp/r6ap; mkdir -p $T
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c2_e2e.py > gpurun_out/r6ap/tests.log 2>&1 || { echo tests failed; tail -8 gpurun_out/r6ap/tests.log; exit 1; }; tail -1 gpurun_out/r6ap/tests.log
CDM_LIB=$R/_ab/head.so timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/a.npz || exit 1
CDM_LIB=$R/_ab/bf.so timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6ap/bitexact.txt
for r in 1 2 3; do
  for L in head bf; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/$L w0: /" | tee -a gpurun_out/r6ap/ab.txt
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$L C2: /" | tee -a gpurun_out/r6ap/ab.txt
  done
done
echo ALL_DONE
