#!/bin/bash
# round 3: PMC passes on the final build (HBM bytes per kernel: FETCH_SIZE / WRITE_SIZE in separate runs;
# the split GEMM's SQ / TCC counters on conv2's shape), summaries for bench.py
set -e
O=gpurun_out/r03_pmc
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline --generation off > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline --generation off > $R/$O/pmc_write.log 2>&1
python3 $R/tools/pmc_summary.py $R/$O/pmc_fetch/run_counter_collection.csv $R/$O/pmc_write/run_counter_collection.csv > $R/$O/pmc_summary.json
v=4
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p1 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p2 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p2.log 2>&1
python3 $R/tools/split_gemm_pmc.py --summary $R/$O/v${v}_p1/run_counter_collection.csv $R/$O/v${v}_p2/run_counter_collection.csv > $R/$O/v${v}_pmc.json
rm -rf $R/$O/pmc_fetch $R/$O/pmc_write $R/$O/v${v}_p1 $R/$O/v${v}_p2
echo done
