# PMC HBM passes over the default bench (FETCH_SIZE, WRITE_SIZE in separate runs) and the
# split GEMM's own counters (conv2 shape), then the summaries bench.py reads.
# usage: bash tools/gpu_pmc.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-pmc}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_write -o run -- python3 $R/bench.py --steps 2 --no-cpu-baseline > $R/$O/pmc_write.log 2>&1
python3 $R/tools/pmc_summary.py $R/$O/pmc_fetch/run_counter_collection.csv $R/$O/pmc_write/run_counter_collection.csv > $R/$O/pmc_summary.json
v=4
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p1 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p2 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p2.log 2>&1
python3 $R/tools/split_gemm_pmc.py --summary $R/$O/v${v}_p1/run_counter_collection.csv $R/$O/v${v}_p2/run_counter_collection.csv > $R/$O/v${v}_pmc.json
cd $R
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
