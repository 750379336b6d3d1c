"""FETCH_SIZE calibration: run under `rocprofv3 --pmc FETCH_SIZE` (tools/gpu.sh
fetch_calib); each dispatch reads a known 1 GiB at 4-, 8- or 16-byte lanes (tools/fetch_calib.hip).
With --summary <counter csv> it prints, per width, FETCH_SIZE x 1024 / bytes read: the factor that
turns the counter into HBM bytes for that access width.

    python tools/fetch_calib.py                       # the dispatches (under rocprofv3)
    python tools/fetch_calib.py --summary run_counter_collection.csv
"""
import csv
import ctypes
import json
import os
import sys

NBYTES = 1 << 30
ORDER = [4, 8, 16] * 3


def run():
    import torch
    L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfetch_calib.so"))
    L.fetch_calib_read.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_void_p]
    x = torch.randint(0, 1 << 20, (NBYTES // 4,), dtype=torch.int32, device="cuda")
    grid = 2048
    out = torch.empty(grid * 4, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    flush = torch.empty(1 << 29, dtype=torch.int32, device="cuda")  # 2 GiB written between dispatches: cold caches
    for w in ORDER:
        flush.fill_(w)
        assert L.fetch_calib_read(ctypes.c_void_p(x.data_ptr()), NBYTES, w, ctypes.c_void_p(out.data_ptr()), grid,
                                  st) == 0
    torch.cuda.synchronize()
    print(json.dumps({"bytes_per_dispatch": NBYTES, "widths_in_order": ORDER}))


def summary(path):
    rows = [r for r in csv.DictReader(open(path)) if "read_kernel" in r["Kernel_Name"]
            and r.get("Counter_Name") == "FETCH_SIZE"]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
    per = {}
    for w, r in zip(ORDER, rows):
        per.setdefault(w, []).append(float(r["Counter_Value"]) * 1024 / NBYTES)
    print(json.dumps({"what": "FETCH_SIZE x 1024 / bytes actually read (1 GiB, every line once, whole)",
                      "source": path, "factor_by_lane_width_bytes": per,
                      "note": "a factor of 0.5 means FETCH_SIZE must be doubled for that width (the gfx950 "
                              "correction); 1.0 means it reports the bytes as they are"}, indent=1))


if __name__ == "__main__":
    if "--summary" in sys.argv:
        summary(sys.argv[sys.argv.index("--summary") + 1])
    else:
        run()
