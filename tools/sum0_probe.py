#!/usr/bin/env python3
"""torch's bf16 batch sum of a (256, 197, 768) tensor, idle and beside a side-stream GEMM, for a
rocprofv3 --kernel-trace: do the two launches differ (kernel, grid), and by how much the results?"""
import json
import torch
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
m = torch.randn(256, 197, 768, device=dev, generator=g).to(torch.bfloat16)
a = torch.randn(50432, 768, device=dev, generator=g).to(torch.bfloat16)
w = torch.randn(3072, 768, device=dev, generator=g).to(torch.bfloat16)
side = torch.cuda.Stream()
ref = m.sum(0, keepdim=True)
torch.cuda.synchronize()
res = []
for it in range(6):
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            torch.nn.functional.linear(a, w)
    got = m.sum(0, keepdim=True)
    f32 = m.sum(0, keepdim=True, dtype=torch.float32)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    idle = m.sum(0, keepdim=True, dtype=torch.float32)
    res.append({"bf16_equal": bool(torch.equal(got, ref)),
                "bf16_maxdiff": float((got.float() - ref.float()).abs().max()),
                "n_diff": int((got != ref).sum()),
                "f32_equal": bool(torch.equal(f32, idle)),
                "f32_maxdiff": float((f32 - idle).abs().max())})
print(json.dumps(res))
