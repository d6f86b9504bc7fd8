# round 3: host-to-kernel-start latency of the first launch after a synchronize
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python -u tools/probes/launch_latency.py > $O/probe.json 2> $O/probe.err || exit 1
python tools/probes/launch_latency_report.py $O/trace $O/probe.json > $O/report.txt || exit 2
find $O -name "run_*.csv" -delete
