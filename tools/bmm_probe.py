import torch, time
def t(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-s)/it
for T in [65536, 36864, 16384]:
    V = torch.randn(16, T, 512, device="cuda"); U = torch.randn(16, 512, 512, device="cuda")
    M = torch.empty(16, T, 512, device="cuda")
    dt = t(lambda: torch.bmm(V, U, out=M))
    fl = 2*16*T*512*512
    print(T, f"{dt*1e3:.3f} ms", f"{fl/dt/1e12:.1f} TF/s", flush=True)
    # also one big matmul [16T,512]x[512,512] for comparison
    V2 = V.reshape(-1, 512)
    dt2 = t(lambda: torch.mm(V2, U[0]))
    print("  mm", f"{dt2*1e3:.3f} ms", f"{fl/dt2/1e12:.1f} TF/s", flush=True)
