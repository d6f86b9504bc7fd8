#!/bin/bash
# One parametrised GPU-box runner (replaces round 3's one-off r03*_run.sh
# scripts, now kept beside their outputs under profiles/r03/scripts/).
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
# Outputs go to gpurun_out/TAG/.  Each STEP runs under its own time limit;
# the first failing step ends the script with its index as the exit status
# (no later GPU step runs after a fault or a timeout).  Steps:
#   gpu_tests               the whole -m gpu suite              -> tests.log
#   pytest=PATHS            these test files / node ids         -> pytest_<i>.log
#   smoke                   __graft_entry__.smoke()             -> smoke.log
#   bench[:LABEL]=ARGS      python bench.py ARGS                -> bench_LABEL.json / .err
#   torchrun1[:LABEL]=ARGS  bench.py under torch.distributed.run, one rank (the driver's N > 1 launch form)
#   nccl_host               tools/nccl_host_cost.py, one RCCL rank -> nccl_host.json
#   profile                 tools/profile.sh TAG (PMC passes + window trace)
#   py[:LABEL]=ARGS         python -u tools/ARGS                -> py_LABEL.log
#   rehearse_n2             tools/rehearse_n2.sh (2 gloo ranks on one GPU)
#   rehearse_n8[=ARGS]      tools/rehearse_n8.sh ARGS (8 gloo ranks on one GPU; ARGS go to bench.py)
#   env=NAME=VALUE          export NAME=VALUE for later steps
#   lib=NAME                later steps load build_variants/liboch_gpu_NAME.so (tools/build_variants.sh);
#                           lib=default goes back to the in-tree library
#   pmc:LABEL=COUNTERS      one rocprofv3 --pmc pass (quote the counter list) over the bench's 20-step
#                           window (BENCH_PMC_ARGS adds bench args) -> pmc_LABEL/, summarised into
#                           pmc_LABEL.json (tools/pmc_summary.py --window); passes of one LABEL accumulate
#   rocpy:LABEL=SCRIPT ARGS rocprofv3 --kernel-trace --stats of python -u tools/SCRIPT ARGS -> roc_LABEL/
#   pmcpy:LABEL=COUNTERS@SCRIPT ARGS   the same pass over python -u tools/SCRIPT ARGS, every dispatch
#                           summarised (no window) -> pmc_LABEL.json
# Example:
#   bash tools/gpu_run.sh r04a pytest=tests/test_gpu_comm.py "bench:sharded=--sharded --no-cpu-baseline" nccl_host
set -o pipefail
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%=*}
  args=""
  [[ "$step" == *=* ]] && args=${step#*=}
  label=${name#*:}
  [[ "$label" == "$name" ]] && label=$i
  base=${name%%:*}
  echo "[$(date +%T)] step $i: $step" >&2
  case "$base" in
    gpu_tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit $i; }
      tail -1 "$O/tests.log" ;;
    pytest)
      timeout -k 10 600 python -u -m pytest $args -m gpu -x -v --timeout 200 --timeout-method thread \
        > "$O/pytest_$i.log" 2>&1 || { tail -40 "$O/pytest_$i.log"; exit $i; }
      tail -1 "$O/pytest_$i.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { tail -20 "$O/smoke.log"; exit $i; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python -u bench.py $args > "$O/bench_$label.json" 2> "$O/bench_$label.err" \
        || { tail -20 "$O/bench_$label.err"; exit $i; }
      python tools/bench_line.py "$O/bench_$label.json" ;;
    torchrun1)
      timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + i)) bench.py $args > "$O/bench_$label.json" 2> "$O/bench_$label.err" \
        || { tail -20 "$O/bench_$label.err"; exit $i; }
      python tools/bench_line.py "$O/bench_$label.json" ;;
    nccl_host)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port $((29500 + i)) tools/nccl_host_cost.py > "$O/nccl_host.json" 2> "$O/nccl_host.err" \
        || { tail -20 "$O/nccl_host.err"; exit $i; }
      cat "$O/nccl_host.json" ;;
    profile)
      bash tools/profile.sh "$TAG" > "$O/profile.log" 2>&1 || { tail -20 "$O/profile.log"; exit $i; } ;;
    py)
      timeout -k 10 600 python -u tools/$args > "$O/py_$label.log" 2>&1 || { tail -20 "$O/py_$label.log"; exit $i; }
      tail -3 "$O/py_$label.log" ;;
    env)
      export "$args" ;;
    lib)
      if [[ "$args" == "default" ]]; then unset OCH_GPU_LIB; else export OCH_GPU_LIB=build_variants/liboch_gpu_$args.so; fi
      [[ -z "$OCH_GPU_LIB" || -f "$OCH_GPU_LIB" ]] || { echo "missing $OCH_GPU_LIB" >&2; exit $i; } ;;
    pmc)
      export TMPDIR=/tmp
      export OCH_TREE_CACHE=${OCH_TREE_CACHE:-/tmp/och_tree_d12.npz}
      timeout -s KILL 240 rocprofv3 --pmc $args --output-format csv -d "$O/pmc_$label/pmc_pass$i" -o run -- \
        python -u bench.py --steps 20 --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce \
        --no-cull-off --moving-steps 0 $BENCH_PMC_ARGS > "$O/pmc_${label}_$i.json" 2> "$O/pmc_${label}_$i.err" \
        || { tail -20 "$O/pmc_${label}_$i.err"; exit $i; }
      python tools/pmc_summary.py "$O/pmc_$label" --window > "$O/pmc_$label.json" || exit $i ;;
    rocpy)
      # rocprofv3 kernel trace (timestamps + per-kernel stats, no counters) of python -u tools/ARGS
      export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/roc_$label" -o run -- \
        python -u tools/$args > "$O/roc_$label.log" 2>&1 || { tail -20 "$O/roc_$label.log"; exit $i; }
      tail -3 "$O/roc_$label.log" ;;
    pmcpy)
      export TMPDIR=/tmp
      counters=${args%%@*}; script=${args#*@}
      timeout -s KILL 240 rocprofv3 --pmc $counters --output-format csv -d "$O/pmc_$label/pmc_pass$i" -o run -- \
        python -u tools/$script > "$O/pmc_${label}_$i.log" 2>&1 || { tail -20 "$O/pmc_${label}_$i.log"; exit $i; }
      python tools/pmc_summary.py "$O/pmc_$label" > "$O/pmc_$label.json" || exit $i ;;
    rehearse_n2)
      bash tools/rehearse_n2.sh > "$O/rehearse_n2.txt" 2>&1 || { tail -20 "$O/rehearse_n2.txt"; exit $i; }
      cp gpurun_out/rehearse_n2.json "$O/" 2>/dev/null ;;
    rehearse_n8)
      bash tools/rehearse_n8.sh $args > "$O/rehearse_n8.txt" 2>&1 || { tail -20 "$O/rehearse_n8.txt"; exit $i; }
      cp gpurun_out/rehearse_n8/bench.json "$O/rehearse_n8.json" 2>/dev/null; tail -c 600 "$O/rehearse_n8.txt" ;;
    *)
      echo "unknown step $step" >&2; exit 100 ;;
  esac
done
echo "[$(date +%T)] done" >&2
