set -o pipefail
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05x_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r05x_tests.log; echo tests_rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05x_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r05x_smoke.log; exit $rc
