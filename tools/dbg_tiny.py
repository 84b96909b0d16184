"""Dev tool: tiny CLIP train-step losses with the mixer glue variants toggled."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mamba-clip_amd"))
import torch
import mamba_clip_amd.model as M
from mamba_clip_amd.loss import ClipLoss

real_nem = M.neg_exp_many
for seed in range(6):
  for hand in (True,):
    for nem in (True,):
        M.neg_exp_many = real_nem if nem else (lambda logs: [None] * len(logs))
        torch.manual_seed(seed)
        model, _, _, _ = M.init_model("tiny-mamba-clip")
        model = model.to("cuda")
        for m in model.modules():
            if hasattr(m, "du_handoff"):
                m.du_handoff = hand
        opt = torch.optim.AdamW(model.parameters(), lr=3e-4)
        g = torch.Generator().manual_seed(seed + 100)
        img = torch.randn(8, 3, 32, 32, generator=g).cuda()
        tok = torch.randint(1, 1000, (8, 16), generator=g).cuda()
        losses = []
        for _ in range(5):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(img, tok)
                loss = ClipLoss()(**out)["contrastive_loss"]
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(round(float(loss), 4))
        print(f"seed {seed} handoff={hand} neg_exp_many={nem}: {losses}", flush=True)
