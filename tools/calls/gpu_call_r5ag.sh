# round 5 (ag): the driver's bench command once more at the final HEAD (box-spread sample) + smoke
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ag_smoke.log 2>&1 || exit 1
echo smoke ok
timeout -k 10 600 python3 bench.py > gpurun_out/r5ag_bench.json 2> gpurun_out/r5ag_bench.err || exit 1
echo bench ok
