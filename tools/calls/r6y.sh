# round 6 (y): the sampling step's per-launch trace at HEAD (w = 0, n = 256; and the CFG 512-image step)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6y
export TMPDIR=/tmp
for w in 0 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6y/w$w -o sample -- \
      python3 tools/sample_profile.py --steps 40 --w $w > gpurun_out/r6y/sample_w$w.log 2> gpurun_out/r6y/sample_w$w.err; echo "prof w=$w rc=$?"
  f=$(ls gpurun_out/r6y/w$w/*kernel_trace.csv | head -1)
  python3 tools/kseg.py $f denoise_kernel 20 > gpurun_out/r6y/kseg_w$w.txt && head -12 gpurun_out/r6y/kseg_w$w.txt
  python3 tools/kstep_list.py $f > gpurun_out/r6y/one_step_w$w.txt; rm -f $f
done
echo ALL_DONE
