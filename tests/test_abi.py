"""The C-ABI boundary without a GPU: libvqx.so loads, exports every function
include/vqx.h declares, its ABI version matches, the ctypes mirrors in
vae_npvc_amd/_lib.py have the header's exact struct layouts (checked against
gcc's own sizeof/offsetof of the header), and argument validation fails
loudly (return code + vqx_last_error) before any device work."""
import ctypes
import re
import subprocess

import pytest

from tests.helpers import ROOT

HEADER = ROOT / "include" / "vqx.h"


def _lib():
    from vae_npvc_amd import _lib as L
    return L, L.load()


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\s*\*)\s+(vqx_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_abi():
    fns = header_functions()
    assert len(fns) >= 28
    for f in ("vqx_conv1d_fwd", "vqx_conv1d_dgrad", "vqx_conv1d_wgrad", "vqx_vq_forward", "vqx_vq_ema_update",
              "vqx_adam_step", "vqx_weight_norm_bwd", "vqx_gn_bwd", "vqx_version", "vqx_last_error"):
        assert f in fns


def test_library_exports_every_header_symbol():
    L, lib = _lib()
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # the Python binding declares a signature for every exported function
    assert set(header_functions()) <= set(L._SIGS) | {"vqx_last_error", "vqx_version"}


def test_abi_version():
    L, lib = _lib()
    assert lib.vqx_version() == L.ABI_VERSION
    m = re.search(r"#define VQX_ABI_VERSION (\d+)", HEADER.read_text())
    assert m and int(m.group(1)) == L.ABI_VERSION


def _c_layout(struct, fields):
    src = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void) {",
           f'  printf("%zu\\n", sizeof({struct}));']
    src += [f'  printf("%zu\\n", offsetof({struct}, {f}));' for f in fields]
    src += ["  return 0;", "}"]
    import tempfile
    import os
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "l.c"), os.path.join(d, "l")
        open(c, "w").write("\n".join(src))
        subprocess.run(["gcc", "-std=c99", "-o", exe, c], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


@pytest.mark.parametrize("struct,cls", [("vqx_conv_args", "ConvArgs"), ("vqx_wgrad_args", "WgradArgs"),
                                        ("vqx_wn_layer", "WNLayer")])
def test_struct_layout_matches_header(struct, cls):
    L, _ = _lib()
    c = getattr(L, cls)
    names = [f[0] for f in c._fields_]
    got = _c_layout(struct, names)
    assert got[0] == ctypes.sizeof(c)
    assert got[1:] == [getattr(c, n).offset for n in names]


def test_validation_errors_are_loud():
    """Bad arguments return -1 with a message; nothing is launched."""
    L, lib = _lib()
    lib.vqx_conv1d_fwd.restype = ctypes.c_int
    lib.vqx_last_error.restype = ctypes.c_char_p
    assert lib.vqx_conv1d_fwd(None, None) != 0
    assert b"null" in lib.vqx_last_error()
    a = L.ConvArgs()
    a.dtype = 7
    assert lib.vqx_conv1d_fwd(ctypes.byref(a), None) != 0
    assert b"dtype" in lib.vqx_last_error()
    a = L.ConvArgs()
    a.dtype, a.ntaps, a.pad, a.n_rows, a.T, a.cin, a.cout, a.ldx, a.ldy = L.VQX_BF16, 3, 1, 100, 64, 512, 512, 512, 512
    assert lib.vqx_conv1d_fwd(ctypes.byref(a), None) != 0  # n_rows not a multiple of T
    assert b"multiple" in lib.vqx_last_error()
    # the Python wrapper raises with the library's message
    with pytest.raises(L.VqxError):
        L.call("vqx_conv1d_fwd", None, None)


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    """The product path has no CPU fallback: without the HIP library it raises."""
    from vae_npvc_amd import _lib as L
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.VqxError):
        L.load(tmp_path / "nope.so")


def test_wgrad_tiles_reports_the_kernel_the_library_picks():
    """vqx_wgrad_tiles is host-only (no GPU): 3-tap pad-1 bf16 layers with
    T % 64 == 0 and c_dim % 64 == 0 get the tap-reuse tiling (128 r x 3 taps x
    64 c), everything else 128 x 128 tiles of the (tap, channel) columns."""
    from vae_npvc_amd import _lib as L
    from vae_npvc_amd import ops
    N, T = 64 * 256, 256
    assert ops.wgrad_tiles(N, T, 512, 512, 3, 1, L.VQX_BF16) == 4 * 8
    assert ops.wgrad_tiles(N, T, 512, 1024, 3, 1, L.VQX_BF16) == 4 * 16
    assert ops.wgrad_tiles(N, T, 512, 512, 1, 0, L.VQX_BF16) == 4 * 4      # 1x1: im2col tiles
    # the call's kernel policy (ABI 125): implicit im2col only -> 128 x 128 tiles of (tap, channel)
    assert ops.wgrad_tiles(N, T, 512, 512, 3, 1, L.VQX_BF16, policy=ops.POLICY_IM2COL) == 4 * 12
    assert ops.wgrad_tiles(N, T, 512, 512, 3, 1, L.VQX_BF16, policy=ops.POLICY_K1_2PCU) == 4 * 8
    assert ops.wgrad_tiles(N, T, 512, 512, 3, 1, L.VQX_F32) == 4 * 12      # fp32 parity mode
    assert ops.wgrad_tiles(N, 100, 512, 512, 3, 1, L.VQX_BF16) == 4 * 12   # T % 64 != 0
    assert ops.wgrad_tiles(N, T, 512, 80, 3, 1, L.VQX_BF16) == 4 * 2       # c_dim % 64 != 0: ceil(240/128)
    with pytest.raises(L.VqxError):
        ops.wgrad_tiles(N, T, 0, 512, 3, 1, L.VQX_BF16)
