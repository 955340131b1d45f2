# round 4 (z): embed weight gradient back to 64x64 tiles; cout1 band kernel thread layout A/B (CDM_COUT1_FULL) on one box
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -k "cout1 or embed or out3 or band or input_grad" tests/ > gpurun_out/r4z_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4z_tests.log
for v in 0 1; do
  CDM_COUT1_FULL=$v bash tools/train_step_profile.sh gpurun_out/r4z_prof_full$v || exit 1
  echo "CDM_COUT1_FULL=$v"; grep -E "steps:|cout1_fwd|embed_bwd_param" gpurun_out/r4z_prof_full$v/breakdown.txt
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z_smoke.txt 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/r4z_smoke.txt
echo ALL_DONE
