# round 3: full GPU suite, smoke, bench N = 1, and the N = 2 path rehearsed with gloo
set -o pipefail
O=gpurun_out/r03ah; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
bash tools/rehearse_n2.sh > $O/rehearse.txt 2>&1 || exit 4
cp gpurun_out/rehearse_n2.json $O/
bash tools/profile.sh r03ah > $O/profile.log 2>&1 || exit 5
