# diagnosis: train bench (graph) then the inference leg alone, each in its own process; the second only when the
# first ended normally or with a Python exception (rc 0/1), never after a fault / abort / time limit
mkdir -p gpurun_out/r06e
timeout -k 10 300 python3 -X faulthandler bench.py --steps 10 --warmup 3 --no-cpu-baseline --stage-check 0 --augment-bench 0 --lscale-steps 0 > gpurun_out/r06e/a.log 2>&1
rc=$?; echo "a rc=$rc" >> gpurun_out/r06e/rc.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -X faulthandler bench.py --infer --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06e/b.log 2>&1
rc=$?; echo "b rc=$rc" >> gpurun_out/r06e/rc.txt
exit $rc
