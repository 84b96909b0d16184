"""Image input path (include/mc_ops.h mc_patch_embed_input) vs the reference's transform restated in
oracle/cpu_model.py: ToTensor + Normalize(OPENAI mean / std) (src/mamba_clip/data.py:47-53, 102-106)
followed by the patch-embed conv's im2col (k = s = P), and the cast the towers' autocast applies."""
import pytest
import torch

from oracle.cpu_model import IMAGE_MEAN, IMAGE_STD, _im2col, to_tensor_normalize

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [(2, 3, 224, 224, 16), (3, 3, 224, 224, 4), (1, 3, 32, 48, 8), (2, 1, 64, 64, 16), (1, 3, 28, 28, 4),
          (0, 3, 32, 32, 16)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                          (torch.float32, torch.float16), (torch.bfloat16, torch.bfloat16),
                                          (torch.bfloat16, torch.float32)])
def test_float_nchw_patches_bit_exact(shape, in_dt, out_dt):
    """A float image: a permutation plus the autocast cast, so bit-exact vs unfold + .to()."""
    from mamba_clip_amd.ops import patch_im2col
    B, C, H, W, P = shape
    img = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(H + P)).to(in_dt)
    ref = _im2col(img.float(), P).to(out_dt) if in_dt == torch.float32 else _im2col(img, P).to(out_dt)
    got = patch_im2col(img.to(DEV), P, out_dt)
    assert got.dtype == out_dt and got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("out_dt", [torch.float32, torch.bfloat16])
def test_uint8_nhwc_normalize_patches(shape, out_dt):
    """Raw decoded images (B, H, W, C) uint8: ToTensor + Normalize + im2col in one pass.  The kernel
    computes x * (1 / (255 std)) + (-mean / std) in fp32 (one FMA); vs the fp64 restatement it is within
    a few fp32 ulps of |x| <= 2.2 (fp32 output), or one bf16 rounding (bf16 output)."""
    from mamba_clip_amd.ops import patch_im2col
    B, C, H, W, P = shape
    img = torch.randint(0, 256, (B, H, W, C), dtype=torch.uint8, generator=torch.Generator().manual_seed(W + C))
    ref = _im2col(to_tensor_normalize(img), P)
    got = patch_im2col(img.to(DEV), P, out_dt).cpu()
    assert got.dtype == out_dt and got.shape == ref.shape
    if B == 0:
        return
    tol = 2e-6 if out_dt == torch.float32 else 2 ** -7
    assert float((got.float() - ref).abs().max()) <= tol * 2.5
    # the extremes of the byte range land on the reference's per-channel bounds
    lo = torch.tensor([-m / s for m, s in zip(IMAGE_MEAN, IMAGE_STD)][:C])
    assert float(got.float().min()) >= float(lo.min()) - 1e-2


def test_towers_accept_raw_uint8_images():
    """ClipModel on raw uint8 NHWC images == ClipModel on the reference-transformed float NCHW batch
    (same weights), both towers' patch embeddings (ViT-B/16 P 16 and VSSM P 4)."""
    from mamba_clip_amd.model import PatchEmbed, PatchEmbed2D
    torch.manual_seed(0)
    img = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8)
    xf = to_tensor_normalize(img).to(DEV)
    for m in (PatchEmbed().to(DEV), PatchEmbed2D(patch_size=4, embed_dim=96).to(DEV)):
        with torch.no_grad():
            a, b = m(img.to(DEV)), m(xf)
            assert a.shape == b.shape
            assert float((a - b).abs().max() / b.abs().max()) < 1e-5
            with torch.autocast("cuda", dtype=torch.bfloat16):
                a16, b16 = m(img.to(DEV)), m(xf)
            assert a16.dtype == torch.bfloat16
            assert float((a16.float() - b16.float()).abs().max() / b16.float().abs().max()) < 2e-2


def test_float_input_gradient_inverse_permutation():
    from mamba_clip_amd.ops import patch_im2col
    img = torch.randn(2, 3, 32, 32, device=DEV, requires_grad=True)
    g = torch.randn(2 * 4 * 4, 3 * 64, device=DEV)
    patch_im2col(img, 8, torch.bfloat16).float().backward(g.bfloat16().float())
    ref = torch.nn.functional.fold(g.bfloat16().float().reshape(2, 16, 192).transpose(1, 2), (32, 32), 8, stride=8)
    assert img.grad.dtype == torch.float32 and torch.equal(img.grad, ref)


def test_patch_input_rejects_bad_arguments():
    from mamba_clip_amd.ops import patch_im2col
    with pytest.raises(RuntimeError, match="multiple of 4"):
        patch_im2col(torch.zeros(1, 30, 30, 3, dtype=torch.uint8, device=DEV), 6)
    with pytest.raises(RuntimeError, match="1 or 3 channels"):
        patch_im2col(torch.zeros(1, 32, 32, 4, dtype=torch.uint8, device=DEV), 16)
    with pytest.raises(RuntimeError, match="dividing H and W"):
        patch_im2col(torch.zeros(1, 3, 36, 32, device=DEV), 16)


def test_host_to_device_loader_on_gpu():
    """Pinned staging + copy stream: every yielded batch equals the dataset's samples, on the consumer stream."""
    from mamba_clip_amd.data import HostToDeviceLoader, IsicShapedDataset
    ds = IsicShapedDataset(48, image_size=32, context_length=8, vocab_size=100, seed=5)
    ld = HostToDeviceLoader(ds, 8, DEV, seed=2)
    for (img, txt, tgt), idx in zip(ld, ld._order()):
        assert img.is_cuda and img.dtype == torch.uint8
        torch.cuda.current_stream().synchronize()
        assert torch.equal(img.cpu(), ds.images[idx]) and torch.equal(txt.cpu(), ds.texts[idx])
        assert torch.equal(tgt.cpu(), ds.targets[idx])


def test_clip_train_step_on_raw_uint8_batches():
    """One ViT-B/16 + Mamba contrastive step fed raw crops: finite loss, image-tower gradients."""
    from types import SimpleNamespace
    from mamba_clip_amd.data import synthetic_batch
    from mamba_clip_amd.loss import ClipLoss
    from mamba_clip_amd.model import build_clip
    from mamba_clip_amd.train import create_optimizer, train_step
    torch.manual_seed(0)
    model = build_clip("vit_b16-mamba130m").to(DEV)
    args = SimpleNamespace(precision="amp_bf16", lr=1e-4, wd=0.2, beta1=0.9, beta2=0.98, eps=1e-6,
                           grad_clip_norm=None, accum_freq=1)
    opt = create_optimizer(model, args)
    img, txt, tgt = synthetic_batch(4, 224, model.text.context_length, model.text.vocab_size, device=DEV,
                                    image_dtype=torch.uint8)
    losses = train_step(model, img, txt, tgt, ClipLoss(), opt, None, args)
    assert torch.isfinite(losses["loss"])
