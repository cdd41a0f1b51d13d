"""L2 request-size calibration for bench.py's roofline.l2 (run under rocprofv3 --pmc
TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum, scripts/gpu_l2_calib.sh): kernels that read a
known number of bytes once, with 16-B loads per lane like k_render_ps's node and
triangle fetches:
  * a coalesced float4 stream (torch sum over a 1 GiB fp32 tensor);
  * a gather of random 16-B granules, each lane one granule (x[idx] on a (N, 4) fp32
    table), the access shape of the traversal's divergent node loads;
then summarise.py-style: bytes read / (TCC_HIT + TCC_MISS) per kernel."""
import torch

torch.manual_seed(0)
dev = torch.device("cuda", 0)
x = torch.ones(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
torch.cuda.synchronize()
for _ in range(3):
    s = x.sum()
torch.cuda.synchronize()
table = torch.ones((1 << 24, 4), dtype=torch.float32, device=dev)  # 256 MiB of 16-B granules
idx = torch.randint(0, 1 << 24, (1 << 24,), device=dev)
for _ in range(3):
    g = table[idx]
torch.cuda.synchronize()
print("sum bytes", x.numel() * 4, "gather bytes read", idx.numel() * 16, "(+ idx", idx.numel() * 8, ")")
