# PMC passes over the split GEMM alone (conv2 shape), both kernel variants, plus the microbench.
# usage: bash tools/gpu_gemm_pmc.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-gemm_pmc}
mkdir -p $O
R=$PWD
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split or winograd" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/split_gemm_bench.json 2> $O/split_gemm_bench.err
cd /tmp
for v in 4; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p1 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/v${v}_p2 -o run -- python3 $R/tools/split_gemm_pmc.py $v 10 > $R/$O/v${v}_p2.log 2>&1
python3 $R/tools/split_gemm_pmc.py --summary $R/$O/v${v}_p1/*counter_collection.csv $R/$O/v${v}_p2/*counter_collection.csv > $R/$O/v${v}_pmc.json
done
