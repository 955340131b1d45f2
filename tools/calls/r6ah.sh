# round 6 (ah): the driver's round-end steps at HEAD — build check of the in-tree library (no rebuild on the box),
# smoke() on cuda:0, and the 2-rank plumbing rehearsal of bench.py on one GPU (gloo, replicas)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r6ah
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6ah/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r6ah/smoke.log
echo ALL_DONE
