# split GEMM tests + microbench (variants in AZG_SG_VARIANTS)
# usage: bash tools/gpu_gemm.sh <outdir under gpurun_out>
set -e
O=gpurun_out/${1:-gemm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py -m gpu -x -q -k "split_gemm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/split_gemm_bench.py > $O/split_gemm_bench.json 2> $O/split_gemm_bench.err
