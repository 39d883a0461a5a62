#!/bin/bash
# One GPU-box lease, parameterized: runs the named steps in order, each under its own time
# limit, and stops at the first failure (no retries: read what it left under gpurun_out/).
#
# usage: RUN=<tag> scripts/gpu_job.sh <step> [<step> ...]
#   steps:
#     tests[=<pytest args>]   GPU suite (default: the whole -m gpu suite)
#     smoke                   __graft_entry__.smoke()
#     bench                   default `python bench.py` (the driver's line)
#     c3 | c4 | c5            bench.py --workload <w>, short (env passes through, e.g. SBAG_*)
#     c4nd                    the C4 shard with real-valued labels (bench.py's nondyadic line)
#     cont                    scripts/bench_continuous.py (C3 shape on continuous features)
#     gbm                     scripts/bench_gbm.py
#     f64probe                scripts/f64_probe.py, serialized, per-level stage times
#     trace_c3 | trace_c5 | trace_c4   rocprofv3 --kernel-trace --stats of the bench command
#     prof_c3 | prof_c5 | prof_c4      trace + separate PMC passes (scripts/profile.sh)
#     fuzz[=<minutes>]        scripts/fuzz_parity.py; fuzzb: --booster; fuzzbig: --big
#     ab:<NAME>=<v1>,<v2>..:<step>    the step once per value of env NAME (A/B inside one box)
# Example:
#   gpurun --timeout 1200 -- 'RUN=r05a bash scripts/gpu_job.sh tests bench trace_c5'
set -u
export TMPDIR=/tmp
RUN=${RUN:-job}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"

summ() {  # one-line summary of a bench JSON line
  tail -1 "$1" | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
r=d.get('roofline',{})
print(d.get('config',{}).get('workload'), 'ms', d.get('ms_per_step'), 'value %.4g' % d.get('value',0),
      'frac', r.get('frac'), 'launch_ms', r.get('avg_launch_ms'), 'bd', d.get('breakdown_ms'),
      'nondyadic', (d.get('nondyadic_labels') or {}).get('ms_per_step'))" || true
}

run_step() {
  local st=$1 tag=$2 rc
  case "$st" in
    tests|tests=*)
      local args="tests -m gpu"
      [ "$st" != tests ] && args="${st#tests=}"
      timeout -k 10 1100 python -u -m pytest $args -x -q --timeout 600 --timeout-method thread \
        > "$OUT/gpu_tests$tag.log" 2>&1
      rc=$?; tail -3 "$OUT/gpu_tests$tag.log"; [ $rc -ne 0 ] && tail -60 "$OUT/gpu_tests$tag.log"
      return $rc ;;
    smoke)
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke$tag.log" 2>&1
      rc=$?; tail -2 "$OUT/smoke$tag.log"; return $rc ;;
    bench)
      timeout -k 10 500 python3 bench.py > "$OUT/bench$tag.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$OUT/bench$tag.log"; summ "$OUT/bench$tag.log"; return $rc ;;
    c3|c4|c5)
      local extra="--steps 3 --warmup 1"
      [ "$st" = c4 ] && extra="--steps 2 --warmup 1"
      timeout -k 10 400 python3 bench.py --workload $st $extra --no-cpu-baseline --no-nondyadic --no-continuous \
        > "$OUT/bench_$st$tag.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$OUT/bench_$st$tag.log"; summ "$OUT/bench_$st$tag.log"; return $rc ;;
    c4nd)
      # the C4 shard with real-valued labels (bench.py's nondyadic line on the c4 workload)
      timeout -k 10 500 python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-continuous \
        --nondyadic-steps 2 > "$OUT/bench_c4nd$tag.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$OUT/bench_c4nd$tag.log"; summ "$OUT/bench_c4nd$tag.log"; return $rc ;;
    nondyadic)
      timeout -k 10 400 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-continuous --nondyadic-steps 3 \
        > "$OUT/bench_nd$tag.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$OUT/bench_nd$tag.log"; summ "$OUT/bench_nd$tag.log"; return $rc ;;
    cont)
      timeout -k 10 400 python3 -u scripts/bench_continuous.py > "$OUT/cont$tag.log" 2>&1
      rc=$?; tail -4 "$OUT/cont$tag.log"; return $rc ;;
    f64probe)
      SBAG_OVERLAP=0 SBAG_LEVEL_TRACE=1 timeout -k 10 300 python3 -u scripts/f64_probe.py > "$OUT/f64probe$tag.log" 2>&1
      rc=$?; grep "f64 level" "$OUT/f64probe$tag.log" | tail -9; tail -1 "$OUT/f64probe$tag.log" | cut -c1-700; return $rc ;;
    gbm)
      timeout -k 10 400 python3 -u scripts/bench_gbm.py > "$OUT/gbm$tag.log" 2>&1
      rc=$?; tail -4 "$OUT/gbm$tag.log"; return $rc ;;
    trace_f64)
      local d="$OUT/trace_f64$tag"
      mkdir -p "$d"
      SBAG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o trace -- \
        python3 scripts/f64_probe.py > "$d/trace.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -20 "$d/trace.log"; return $rc; }
      tail -1 "$d/trace.log" | cut -c1-400
      f=$(find "$d" -name "*kernel_stats.csv" | head -1); head -20 "$f" | cut -d, -f1-5 | cut -c1-160
      return 0 ;;
    pmc_cont|pmc_f64)
      # two PMC passes (one counter block set each, no trace domains) of the continuous bench /
      # the f64 probe: issue mix and LDS behaviour
      local d="$OUT/$st$tag" cmd="python3 scripts/bench_continuous.py"
      [ "$st" = pmc_f64 ] && cmd="python3 scripts/f64_probe.py"
      mkdir -p "$d"
      timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
        --output-format csv -d "$d/p1" -o p1 -- $cmd > "$d/p1.log" 2>&1 || { tail -5 "$d/p1.log"; return 1; }
      timeout -s KILL 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
        --output-format csv -d "$d/p2" -o p2 -- $cmd > "$d/p2.log" 2>&1 || { tail -5 "$d/p2.log"; return 1; }
      return 0 ;;
    trace_cont)
      local d="$OUT/trace_cont$tag"
      mkdir -p "$d"
      SBAG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o trace -- \
        python3 scripts/bench_continuous.py > "$d/trace.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -20 "$d/trace.log"; return $rc; }
      tail -1 "$d/trace.log" | cut -c1-600
      f=$(find "$d" -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -d, -f1-5 | cut -c1-160
      return 0 ;;
    trace_c3|trace_c4|trace_c5)
      local w=${st#trace_} d="$OUT/trace_${st#trace_}$tag"
      mkdir -p "$d"
      SBAG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o trace -- \
        python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-nondyadic --no-continuous > "$d/trace.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && { tail -20 "$d/trace.log"; return $rc; }
      f=$(find "$d" -name "*kernel_stats.csv" | head -1); head -16 "$f" | cut -d, -f1-5 | cut -c1-160
      return 0 ;;
    prof_c3|prof_c4|prof_c5)
      local w=${st#prof_}
      bash scripts/profile.sh "${RUN}_$w$tag" --workload $w --no-nondyadic; return $? ;;
    fuzz|fuzz=*|fuzzb|fuzzbig)
      local m=3 flag="" start=$((RANDOM * 3 + 100000))
      case "$st" in fuzz=*) m=${st#fuzz=} ;; fuzzb) m=1; flag=--booster ;; fuzzbig) m=3; flag="--big" ;; esac
      timeout -k 10 $((m * 60 + 120)) python3 -u scripts/fuzz_parity.py --minutes $m --start $start $flag \
        > "$OUT/$st$tag.log" 2>&1
      rc=$?; tail -1 "$OUT/$st$tag.log"; [ $rc -ne 0 ] && grep -v "^ok" "$OUT/$st$tag.log" | head -20 | cut -c1-250
      return $rc ;;
    ab:*)
      local spec=${st#ab:} name vals inner v
      name=${spec%%=*}; spec=${spec#*=}; vals=${spec%%:*}; inner=${spec#*:}
      for v in ${vals//,/ }; do
        echo "== $name=$v $inner"
        # (a value may carry more settings: ab:A=1,0+B=1:step runs A=1, then A=0 B=1)
        local first=${v%%+*} more="" tagv=${v//[+=]/_}
        [ "$v" != "$first" ] && more=${v#*+}
        env "$name=$first" ${more//+/ } bash -c "$(declare -f summ run_step); OUT='$OUT' RUN='$RUN'; run_step '$inner' '_${name}_$tagv'" || return $?
      done
      return 0 ;;
    *) echo "unknown step $st"; return 2 ;;
  esac
}

for st in "$@"; do
  echo "== step $st"
  run_step "$st" "" || { echo "step $st failed rc=$?"; exit 1; }
done
echo "gpu_job $RUN done"
