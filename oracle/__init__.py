"""CPU oracle for the mamba-clip hot path -- TEST INFRASTRUCTURE ONLY.

Nothing in the product (``mamba-clip_amd/``) imports this package.  Only
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may use it, and only as the checker / the timed CPU baseline.

Contents
--------
scan_ref.py   restatement of the selective-scan reference semantics that the
              reference embeds at model.py:83-169 (inside
              ``flops_selective_scan_ref``); forward in plain torch-CPU,
              backward by autograd on that restatement.
loss_ref.py   restatement of ClipLoss / all_gather / cross_entropy_loss
              (loss.py:6-147).
models_ref.py fp32 torch-CPU restatement of the encoder towers the build
              defines (ViT-B/16 visual, Mamba text), used to check the
              product modules on identical random weights.

Pinning (see DESIGN.md "Oracle"):
* scan_ref is pinned against golden vectors produced by EXECUTING the
  reference's own embedded selective_scan_ref text (tests/golden/make_golden.py
  extracts it from /root/reference at generation time; the text is not kept in
  this repo).  The upstream CUDA kernel (third-party ``mamba_ssm``, version
  unpinned, absent here) is not available, so bitwise-upstream parity is
  "parity unpinned"; parity is to the reference's reference semantics.
* loss_ref is pinned against golden vectors from importing the reference's
  loss.py as-is (single process and gloo world sizes 2 and 4).
* models_ref: the reference's encoders come from open_clip / HF hub (absent
  offline) -- "parity unpinned" beyond the glue pinned by the SS2D fixtures.
"""
