import torch, time
n = 195_000_000
a = torch.empty(n, dtype=torch.float32, device="cuda"); b = torch.empty_like(a)
a.fill_(1.0)
for _ in range(3): b.copy_(a)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10): b.copy_(a)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 10
print(f"copy 780MB: {dt*1e3:.3f} ms, {2*n*4/dt/1e12:.2f} TB/s")
