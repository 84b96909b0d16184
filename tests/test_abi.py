"""CPU-side checks of the C ABI: the library loads, exports every entry point
include/*.h declares, and the ctypes struct mirrors match the C layout
(offsets computed by compiling the header with gcc).  No GPU calls."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT

INCLUDE = os.path.join(ROOT, "include")


def _declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        if h.endswith(".h"):
            txt = open(os.path.join(INCLUDE, h)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            names |= set(re.findall(r"\b(mc_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_loads_and_exports_every_declared_symbol():
    from mamba_clip_amd import _lib
    lib = _lib.load()
    declared = _declared_functions()
    assert declared, "no declarations found"
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    assert set(declared) <= set(_lib.SYMBOLS), "ctypes SYMBOLS table out of date"
    assert lib.mc_version().startswith(b"mamba_clip_amd")


def test_host_only_entry_points():
    from mamba_clip_amd import _lib
    lib = _lib.load()
    C = _lib.MC_SCAN_CHUNK          # saved-state granularity (32 positions, include/mc_scan.h)
    assert lib.mc_scan_n_chunks(0) == 0
    assert lib.mc_scan_n_chunks(1) == 1
    assert lib.mc_scan_n_chunks(C) == 1
    assert lib.mc_scan_n_chunks(C + 1) == 2
    assert lib.mc_scan_n_chunks(4096) == 4096 // C
    assert lib.mc_scan_chunk_states_bytes(2, 3, 77, 16) == 2 * 3 * ((77 + C - 1) // C) * 16 * 4


def test_validation_errors_without_launch():
    """Bad shapes are rejected on the host before any launch (no GPU needed)."""
    from mamba_clip_amd import _lib
    lib = _lib.load()
    p = _lib.ScanFwdParams()
    p.batch, p.dim, p.seqlen, p.dstate, p.n_groups = 1, 6, 8, 16, 4   # dim % groups != 0
    rc = lib.mc_scan_fwd(ctypes.byref(p), None)
    assert rc == -3 and b"n_groups" in lib.mc_last_error()
    p.n_groups, p.dstate = 1, 999
    assert lib.mc_scan_fwd(ctypes.byref(p), None) == -3
    p.dstate, p.itype = 16, 7
    assert lib.mc_scan_fwd(ctypes.byref(p), None) == -2
    p.itype = 0
    assert lib.mc_scan_fwd(ctypes.byref(p), None) == -1   # null pointers
    with pytest.raises(RuntimeError, match="mc_scan_fwd"):
        _lib.check(lib.mc_scan_fwd(ctypes.byref(p), None), "mc_scan_fwd")


def test_wgrad_validation_without_launch():
    """mc_gemm_wgrad rejects bad shapes / layouts on the host; workspace sizing is host-only."""
    from mamba_clip_amd import _lib
    lib = _lib.load()
    p = _lib.WgradParams()
    p.M, p.N, p.T, p.dtype = 768, 768, 100, _lib.MC_DTYPE_BF16        # T % 64 != 0
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -3 and b"multiple of 64" in lib.mc_last_error()
    p.T, p.dtype = 50432, _lib.MC_DTYPE_F32
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -2
    p.dtype, p.a_layout = _lib.MC_DTYPE_BF16, 7
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -1
    p.a_layout = _lib.MC_WGRAD_TOKEN_MAJOR
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -3             # null operands
    p.A = p.B = p.C = 4096
    p.lda = p.ldb = 768
    p.ldc = 769
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -3 and b"contiguous" in lib.mc_last_error()
    p.ldc = 768
    # 9 output tiles of 256 x 256 -> about one workgroup per CU: 28 splits of fp32 slabs
    assert lib.mc_gemm_wgrad_workspace_bytes(ctypes.byref(p)) == 28 * 768 * 768 * 4
    p.splits = 1
    assert lib.mc_gemm_wgrad_workspace_bytes(ctypes.byref(p)) == 0
    p.splits = 0
    p.workspace, p.workspace_bytes = 4096, 16
    assert lib.mc_gemm_wgrad(ctypes.byref(p), None) == -5             # workspace too small


def test_fused_ce_validation_without_launch():
    """mc_ce_fused_fwd / _grad reject bad arguments on the host."""
    from mamba_clip_amd import _lib
    lib = _lib.load()
    p = _lib.CEFusedParams()
    p.M, p.N, p.K, p.in_dtype = 4, 4, 8, _lib.MC_DTYPE_BF16
    assert lib.mc_ce_fused_fwd(ctypes.byref(p), None) == -1 and b"null operand" in lib.mc_last_error()
    p.X = p.Y = 4096
    p.in_dtype = 9
    assert lib.mc_ce_fused_fwd(ctypes.byref(p), None) == -2
    p.in_dtype, p.row_off = _lib.MC_DTYPE_BF16, 1 << 31
    assert lib.mc_ce_fused_fwd(ctypes.byref(p), None) == -3
    p.row_off = 0
    assert lib.mc_ce_fused_fwd(ctypes.byref(p), None) == -1          # null lse_r / loss_out
    p.lse_r = p.loss_out = 4096
    assert lib.mc_ce_fused_fwd(ctypes.byref(p), None) == -5          # no workspace
    assert lib.mc_ce_fused_grad(ctypes.byref(p), None) == -1         # null G
    p.lse_r = None
    assert lib.mc_ce_fused_grad(ctypes.byref(p), None) == -1 and b"both NULL" in lib.mc_last_error()
    assert lib.mc_ce_fused_fwd_workspace_bytes(8192, 8192, 1) < 8192 * 8192   # O(N^2 / 128), not N^2
    assert lib.mc_ce_fused_fwd_workspace_bytes(0, 5, 1) == 0


def test_attention_validation_without_launch():
    """mc_attn_fwd / _bwd reject unsupported shapes, dtypes and layouts on the host."""
    from mamba_clip_amd import _lib
    lib = _lib.load()
    p = _lib.AttnFwdParams()
    p.batch, p.heads, p.seqlen, p.head_dim, p.dtype = 2, 12, 197, 128, _lib.MC_DTYPE_BF16
    assert lib.mc_attn_fwd(ctypes.byref(p), None) == -3 and b"head_dim" in lib.mc_last_error()
    p.head_dim, p.seqlen = 64, 257
    assert lib.mc_attn_fwd(ctypes.byref(p), None) == -3
    p.seqlen, p.dtype = 197, _lib.MC_DTYPE_F32
    assert lib.mc_attn_fwd(ctypes.byref(p), None) == -2
    p.dtype = _lib.MC_DTYPE_BF16
    assert lib.mc_attn_fwd(ctypes.byref(p), None) == -1          # null tensors
    p.q = p.k = p.v = p.o = p.lse = 4096
    p.q_bs, p.q_ns, p.q_hs, p.o_bs, p.o_ns, p.o_hs = 197 * 2304, 2304, 64, 197 * 768, 770, 64   # o_ns % 8 != 0
    assert lib.mc_attn_fwd(ctypes.byref(p), None) == -1 and b"aligned" in lib.mc_last_error()
    b = _lib.AttnBwdParams()
    b.batch, b.heads, b.seqlen, b.head_dim, b.dtype = 2, 12, 197, 64, _lib.MC_DTYPE_BF16
    assert lib.mc_attn_bwd(ctypes.byref(b), None) == -1


@pytest.mark.parametrize("cname,pyname", [("mc_scan_fwd_params", "ScanFwdParams"),
                                          ("mc_scan_bwd_params", "ScanBwdParams"),
                                          ("mc_gemm_nt_params", "GemmNTParams"),
                                          ("mc_ce_fused_params", "CEFusedParams"),
                                          ("mc_qkv_pack_params", "QkvPackParams"),
                                          ("mc_attn_fwd_params", "AttnFwdParams"),
                                          ("mc_attn_bwd_params", "AttnBwdParams"),
                                          ("mc_ss2d_conv_params", "SS2DConvParams"),
                                          ("mc_ss2d_conv_bwd_params", "SS2DConvBwdParams"),
                                          ("mc_ss2d_merge_params", "SS2DMergeParams"),
                                          ("mc_ss2d_merge_bwd_params", "SS2DMergeBwdParams"),
                                          ("mc_patch_input_params", "PatchInputParams"),
                                          ("mc_mixer_proj_params", "MixerProjParams"),
                                          ("mc_mixer_proj_bwd_params", "MixerProjBwdParams"),
                                          ("mc_wgrad_params", "WgradParams")])
def test_struct_layout_matches_header(cname, pyname):
    from mamba_clip_amd import _lib
    cls = getattr(_lib, pyname)
    fields = [f for f, _ in cls._fields_]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "mc_scan.h"', '#include "mc_contrastive.h"',
           '#include "mc_ops.h"', '#include "mc_attn.h"', '#include "mc_ss2d.h"', '#include "mc_gemm.h"',
           "int main(void){",
           f'printf("size %zu\\n", sizeof({cname}));']
    src += [f'printf("{f} %zu\\n", offsetof({cname}, {f}));' for f in fields]
    src += ["return 0;}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", INCLUDE, c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = dict(line.split() for line in out if line)
    assert int(got["size"]) == ctypes.sizeof(cls)
    for f in fields:
        assert int(got[f]) == getattr(cls, f).offset, f


def test_cast_chunk_layout_matches_python_table():
    """ops._CastPlan builds the mc_cast_f32_many chunk table as int64 triples (src, dst_off, n):
    mc_cast_chunk must be 24 B with fields at 0 / 8 / 16."""
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "mc_ops.h"', "int main(void){",
           'printf("%zu %zu %zu %zu\\n", sizeof(mc_cast_chunk), offsetof(mc_cast_chunk, src), '
           'offsetof(mc_cast_chunk, dst_off), offsetof(mc_cast_chunk, n));', "return 0;}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", INCLUDE, c, "-o", exe])
        assert subprocess.check_output([exe]).decode().split() == ["24", "0", "8", "16"]


def test_cast_transpose_tile_layout_matches_python_table():
    """ops._TransposePlan packs each mc_cast_t_tile as four int64: src, dst_off, src_ld | dst_ld << 32,
    rows | cols << 32 (little endian): the struct must be 32 B with fields at 0 / 8 / 16 / 20 / 24 / 28."""
    f = ["src", "dst_off", "src_ld", "dst_ld", "rows", "cols"]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "mc_ops.h"', "int main(void){",
           'printf("%zu", sizeof(mc_cast_t_tile));'] + \
          [f'printf(" %zu", offsetof(mc_cast_t_tile, {n}));' for n in f] + ['printf("\\n");', "return 0;}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", INCLUDE, c, "-o", exe])
        assert subprocess.check_output([exe]).decode().split() == ["32", "0", "8", "16", "20", "24", "28"]


def test_adamw_tables_match_python_layout():
    """optim.HipAdamW packs mc_adamw_chunk as int64 (tensor | group << 32, off, n) and mc_adamw_tensor as
    four pointers; _lib.AdamWHyper mirrors mc_adamw_hyper (passed by pointer, read by value)."""
    from mamba_clip_amd import _lib
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "mc_ops.h"', "int main(void){",
           'printf("%zu %zu %zu %zu %zu ", sizeof(mc_adamw_chunk), offsetof(mc_adamw_chunk, tensor), '
           'offsetof(mc_adamw_chunk, group), offsetof(mc_adamw_chunk, off), offsetof(mc_adamw_chunk, n));',
           'printf("%zu %zu ", sizeof(mc_adamw_tensor), offsetof(mc_adamw_tensor, g));',
           'printf("%zu %zu %zu\\n", sizeof(mc_adamw_hyper), offsetof(mc_adamw_hyper, group), sizeof(mc_adamw_group));',
           "return 0;}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write("\n".join(src))
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", INCLUDE, c, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).decode().split()]
    assert got[:5] == [24, 0, 4, 8, 16] and got[5:7] == [32, 24]
    assert got[7] == ctypes.sizeof(_lib.AdamWHyper) and got[8] == _lib.AdamWHyper.group.offset
    assert got[9] == ctypes.sizeof(_lib.AdamWGroup)
