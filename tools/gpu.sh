#!/bin/bash
# The one GPU-box runner (replaces the per-round gpu_*.sh launchers).
#
#   bash tools/gpu.sh <run-name> <task> [<task> ...]
#
# Output goes to <repo>/gpurun_out/<run-name>/ (paths resolved from this script's own
# directory, never from the caller's cwd; nothing is deleted outside that directory).
# Tasks run in order; the first failing task ends the run (set -e), and every GPU step has
# its own time limit.
#
#   suite               pytest -m gpu (whole suite) -> pytest_gpu.log
#   smoke               __graft_entry__.smoke()     -> smoke.log
#   test:<path>[:<k>]   pytest -m gpu on one file, optionally -k <k> -> test_<file>.log
#   bench[:<args>]      python bench.py <args> (commas become spaces) -> bench[_<tag>].json / .err
#   prof[:<args>]       rocprofv3 --kernel-trace --stats over bench.py <args> (summary prof[_<tag>].md)
#   pmc                 FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 -> pmc_summary.json
#   trace[:<args>]      rocprofv3 --kernel-trace over bench.py <args>, kept; per-launch summaries of
#                       winograd_first and the persistent split GEMM (tools/trace_summary.py)
#   gemm_pmc[:<v>]      split-GEMM SQ/TCC counters on conv2's shape (variant v, default 4) -> v<v>_pmc.json
#   configs             bench.py over C1 / C2 (full games, eager + graph) / C3 / C5 / C4 full games
#   py:<script>[:<args>] python <script> <args> -> <script base>.out / .err
#   profpy:<script>[:<args>] rocprofv3 --kernel-trace --stats over python <script> <args> -> prof_<base>.md
set -e
FAILED=0
R=$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)
NAME=${1:?usage: tools/gpu.sh <run-name> <task> ...}
shift
O=$R/gpurun_out/$NAME
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"

tag_of() {  # a file-name tag for an argument string
    echo "$1" | tr -c 'A-Za-z0-9\n' '_' | sed 's/__*/_/g; s/^_//; s/_$//'
}

for task in "$@"; do
    kind=${task%%:*}
    arg=""
    [[ "$task" == *:* ]] && arg=${task#*:}
    echo "== $task ($(date +%T))"
    case "$kind" in
    suite)
        # no -x: one run lists every failing test; exit 1 (assertion failures only) lets the run go on
        rc=0
        timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rf --timeout 170 --timeout-method thread \
            --durations 15 > "$O/pytest_gpu.log" 2>&1 || rc=$?
        if [ $rc -ne 0 ]; then
            echo "   suite: pytest exit $rc"
            if [ $rc -ne 1 ] || grep -qi "hipError\|memory access fault\|illegal address\|HSA_STATUS" "$O/pytest_gpu.log"; then
                exit $rc
            fi
            FAILED=1
        fi ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    test)
        path=${arg%%:*}
        k=""
        [[ "$arg" == *:* ]] && k=${arg#*:}
        log="$O/test_$(basename "$path" .py)"
        if [ -n "$k" ]; then log="${log}_$(tag_of "$k")"; fi
        log="$log.log"
        kk=()
        [ -n "$k" ] && kk=(-k "$k")
        rc=0
        timeout -k 10 1100 python -u -m pytest "$path" -m gpu -v -s --timeout 170 --timeout-method thread \
            --durations 10 "${kk[@]}" > "$log" 2>&1 || rc=$?
        # exit 1 = assertion failures only: the run goes on to its other tasks unless the log shows
        # a device error; any other status (abort, fault, time limit) ends the run here
        if [ $rc -ne 0 ]; then
            echo "   $path: pytest exit $rc"
            if [ $rc -ne 1 ] || grep -qi "hipError\|memory access fault\|illegal address\|HSA_STATUS" "$log"; then
                exit $rc
            fi
            FAILED=1
        fi ;;
    bench)
        a=${arg//,/ }
        t=$(tag_of "$a")
        timeout -k 10 600 python -u bench.py $a > "$O/bench${t:+_$t}.json" 2> "$O/bench${t:+_$t}.err" ;;
    prof)
        a=${arg//,/ }
        t=$(tag_of "$a")
        d="$O/prof${t:+_$t}"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
            -- python3 "$R/bench.py" $a > "$d.json" 2> "$d.err")
        python3 tools/prof_summary.py "$d/run_kernel_stats.csv" > "$d.md"
        rm -f "$d"/*trace*.csv ;;
    fetch_calib)
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_calib" -o run \
            -- python3 "$R/tools/fetch_calib.py" > "$O/fetch_calib.log" 2>&1)
        python3 tools/fetch_calib.py --summary "$O/fetch_calib/run_counter_collection.csv" > "$O/fetch_calib.json" ;;
    trace)
        # kernel trace kept (per-launch durations and neighbours): tools/trace_summary.py <csv> <kernel>
        a=${arg//,/ }
        t=$(tag_of "$a")
        d="$O/trace${t:+_$t}"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run \
            -- python3 "$R/bench.py" $a > "$d.json" 2> "$d.err")
        python3 tools/trace_summary.py "$d/run_kernel_trace.csv" winograd_first > "$d.first.json"
        python3 tools/trace_summary.py "$d/run_kernel_trace.csv" split_gemm_persist > "$d.gemm.json" ;;
    pmc)
        # pmc[:<bench args>] (default: the C4 line, 2 steps); no generation / learn-iteration pass
        a=${arg//,/ }
        t=$(tag_of "$a")
        [ -z "$a" ] && a="--steps 2"
        (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc${t:+_$t}_fetch" -o run \
            -- python3 "$R/bench.py" $a --no-cpu-baseline --generation off --learn-iteration off \
            > "$O/pmc${t:+_$t}_fetch.log" 2>&1)
        (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc${t:+_$t}_write" -o run \
            -- python3 "$R/bench.py" $a --no-cpu-baseline --generation off --learn-iteration off \
            > "$O/pmc${t:+_$t}_write.log" 2>&1)
        python3 tools/pmc_summary.py "$O/pmc${t:+_$t}_fetch/run_counter_collection.csv" \
            "$O/pmc${t:+_$t}_write/run_counter_collection.csv" > "$O/pmc${t:+_$t}_summary.json" ;;
    gemm_pmc)
        v=${arg:-4}
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
            --output-format csv -d "$O/v${v}_p1" -o run -- python3 "$R/tools/split_gemm_pmc.py" $v 10 \
            > "$O/v${v}_p1.log" 2>&1)
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS \
            GRBM_GUI_ACTIVE --output-format csv -d "$O/v${v}_p2" -o run -- python3 "$R/tools/split_gemm_pmc.py" $v 10 \
            > "$O/v${v}_p2.log" 2>&1)
        python3 tools/split_gemm_pmc.py --summary "$O/v${v}_p1/run_counter_collection.csv" \
            "$O/v${v}_p2/run_counter_collection.csv" > "$O/v${v}_pmc.json" ;;
    configs)
        for c in C1 C3 C5; do
            timeout -k 10 300 python -u bench.py --config $c > "$O/bench_$c.json" 2> "$O/bench_$c.err"
        done
        timeout -k 10 300 python -u bench.py --config C1 --full-games --graph --no-cpu-baseline \
            > "$O/bench_C1_full_graph.json" 2> "$O/bench_C1_full_graph.err"
        timeout -k 10 300 python -u bench.py --config C2 --full-games --no-cpu-baseline \
            > "$O/bench_C2_full.json" 2> "$O/bench_C2_full.err"
        timeout -k 10 300 python -u bench.py --config C2 --full-games --graph --no-cpu-baseline \
            > "$O/bench_C2_full_graph.json" 2> "$O/bench_C2_full_graph.err"
        timeout -k 10 300 python -u bench.py --full-games --no-cpu-baseline \
            > "$O/bench_C4_full.json" 2> "$O/bench_C4_full.err" ;;
    py)
        script=${arg%%:*}
        a=""
        [[ "$arg" == *:* ]] && a=${arg#*:}
        a=${a//,/ }
        b=$(basename "$script" .py)
        timeout -k 10 600 python -u "$script" $a > "$O/$b.out" 2> "$O/$b.err" ;;
    profpy)
        script=${arg%%:*}
        a=""
        [[ "$arg" == *:* ]] && a=${arg#*:}
        a=${a//,/ }
        b=$(basename "$script" .py)
        d="$O/prof_$b"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
            -- python3 "$R/$script" $a > "$d.out" 2> "$d.err")
        python3 tools/prof_summary.py "$d/run_kernel_stats.csv" > "$d.md"
        rm -f "$d"/*trace*.csv ;;
    *)
        echo "unknown task $task" >&2
        exit 2 ;;
    esac
done
echo "== done ($(date +%T))"
exit ${FAILED:-0}
