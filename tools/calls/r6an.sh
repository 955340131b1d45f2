# round 6 (an): the B-early halo schedule as a compile-time constant (no runtime switch: one gload_b site per chunk, 11
# fewer SALU / 3 fewer vmem instructions in the eval chunk loop) vs the runtime-switched build — bit-exactness and
# same-box A/B (sampling, C2)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6an; T=/tmp/r6an; mkdir -p $T
CDM_LIB=$R/_ab/head.so timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/a.npz || exit 1
CDM_LIB=$R/_ab/ce.so timeout -k 10 200 python3 tools/tall_check.py --math h3 --out $T/b.npz || exit 1
python3 tools/tall_check.py --cmp $T/a.npz $T/b.npz | tee gpurun_out/r6an/bitexact.txt
for r in 1 2 3; do
  for L in head ce; do
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/sample_profile.py --steps 200 2>/dev/null | tail -1 | sed "s/^/$L w0: /" | tee -a gpurun_out/r6an/ab.txt
    CDM_LIB=$R/_ab/$L.so timeout -k 10 200 python3 tools/train_profile.py --math h3 --steps 10 --warmup 3 2>/dev/null | tail -1 | sed "s/^/$L C2: /" | tee -a gpurun_out/r6an/ab.txt
  done
done
echo ALL_DONE
