# l-scale per-conv-site table (sorted by time above the attainable roofline) + wgrad micro at l-scale P3 shapes
mkdir -p gpurun_out/r06t
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 scripts/conv_table.py --scale l --img 1280 --bs 16 --steps 1 --by-gap --top 60 > gpurun_out/r06t/l_table.txt 2>&1 &&
timeout -k 10 200 python3 scripts/conv_table.py --bs 64 --steps 2 --by-gap --top 60 > gpurun_out/r06t/n_table.txt 2>&1 &&
for sh in "16 160 160 256 256 3 3 1" "16 160 160 256 256 1 1 1" "16 80 80 512 512 3 3 1" "16 320 320 128 128 3 3 1" "16 320 320 128 256 3 3 2"; do
  timeout -k 10 60 python3 scripts/conv_micro.py wgrad $sh 10 >> gpurun_out/r06t/micro.txt 2>&1 || exit 1
  timeout -k 10 60 python3 scripts/conv_micro.py fwd2 $sh 10 >> gpurun_out/r06t/micro.txt 2>&1 || exit 1
done
