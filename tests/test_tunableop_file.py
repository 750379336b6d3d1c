"""The packaged TunableOp results (nnet.TUNABLEOP_RESULTS, written by tools/tune_gemms.py on an MI355X):
TunableOp's validator header for this image's gfx950, and a solution for every FC GEMM of the training
step at the reference's 512-example batch and the data-parallel trainer's 256 / 128 / 64-example slices."""
import azg_amd  # noqa: F401
from azg_amd import nnet


def _rows():
    with open(nnet.TUNABLEOP_RESULTS) as f:
        return [line.rstrip("\n").split(",") for line in f if line.strip()]


def test_validators():
    val = {r[1]: r[2] for r in _rows() if r[0] == "Validator"}
    for key in ("PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"):
        assert key in val
    assert val["GCN_ARCH_NAME"].startswith("gfx950")


def test_fc_shapes_covered():
    params = {r[1] for r in _rows() if r[0] != "Validator"}
    for b in (512, 256, 128, 64):
        # fc1 forward (4608 -> 1024 on b examples) and fc2 forward (1024 -> 512), both with bias
        assert f"tn_1024_{b}_4608_ld_4608_4608_1024" in params
        assert f"tn_512_{b}_1024_ld_1024_1024_512" in params
    for r in _rows():
        if r[0] != "Validator":
            assert len(r) == 4 and float(r[3]) > 0.0
