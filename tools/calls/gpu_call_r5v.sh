# round 5 (v): the sampling step's kernel trace at HEAD — per-family and per-launch times of one denoise step
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5v
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5v -o sample -- \
    python3 tools/sample_profile.py --steps 40 > gpurun_out/r5v/sample.log 2> gpurun_out/r5v/sample.err; echo "prof rc=$?"
f=$(ls gpurun_out/r5v/*kernel_trace.csv | head -1)
python3 tools/kseg.py $f denoise_kernel 20 > gpurun_out/r5v/kseg.txt && cat gpurun_out/r5v/kseg.txt
python3 - "$f" > gpurun_out/r5v/one_step.txt <<'PY'
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "denoise_kernel" in r["Kernel_Name"]]
seg = rows[idx[-3] + 1: idx[-2] + 1]
for r in seg:
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("cdm::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{d:9.1f} us grid {r.get('Grid_Size_X', r.get('Grid_Size',''))} wg {r.get('Workgroup_Size_X', r.get('Workgroup_Size',''))} {n[:120]}")
PY
cat gpurun_out/r5v/one_step.txt; rm -f $f
echo ALL_DONE
