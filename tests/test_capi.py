"""The C-ABI library loads and exports every symbol include/wgaead.h declares;
struct layouts match the header; without a device every entry point fails
loudly (no CPU fallback). No GPU compute here."""
import ctypes
import os
import re
import subprocess

import pytest

from wgtest import ROOT, wg

HEADER = os.path.join(ROOT, "include/wgaead.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(wg_[a-z0-9_]+)\(", src, re.M)))


def test_header_declares_api():
    names = declared_functions()
    for must in ["wg_seal_batch", "wg_open_batch", "wg_aead_batch", "wg_seal1", "wg_open1", "wg_keys_set",
                 "wg_keys_zero", "wg_ctx_create", "wg_ctx_destroy", "wg_aead_selftest"]:
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = wg().lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    bound = {name for name, _, _ in wg()._lib.SIGNATURES}
    assert set(declared_functions()) == bound


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "wgaead.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(wg_pkt), offsetof(wg_pkt, len),'
                   ' offsetof(wg_pkt, key_slot), sizeof(wg_aead_desc), offsetof(wg_aead_desc, nonce),'
                   ' offsetof(wg_aead_desc, ctr0));'
                   ' printf("%zu %zu %zu %zu %zu\\n", sizeof(wg_batch), offsetof(wg_batch, status),'
                   ' offsetof(wg_batch, in_size), offsetof(wg_batch, n), offsetof(wg_batch, flags)); return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    L = wg()._lib
    assert got == [ctypes.sizeof(L.WgPkt), L.WgPkt.len.offset, L.WgPkt.key_slot.offset, ctypes.sizeof(L.WgAeadDesc),
                   L.WgAeadDesc.nonce.offset, L.WgAeadDesc.ctr0.offset, ctypes.sizeof(L.WgBatch),
                   L.WgBatch.status.offset, L.WgBatch.in_size.offset, L.WgBatch.n.offset, L.WgBatch.flags.offset]
    assert wg().WG_PKT_DTYPE.itemsize == 32


def test_version_string():
    assert b"gfx950" in wg().lib().wg_version()


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure path")
def test_no_device_fails_loudly():
    W = wg()
    with pytest.raises(W.WgError) as e:
        W.Engine(0, 4)
    assert e.value.code == W._lib.WG_EDEVICE
    assert W.lib().wg_aead_selftest(0) == 0


def test_desc_packing_matches_c_layout():
    import numpy as np
    W = wg()
    d = W.pack_desc([1, 2], [3, 4], [5, (1 << 64) - 1], [1420, 0], [7, 8])
    q = W.desc_as_int64(d)
    assert q.shape == (2, 4)
    assert q[0].tolist() == [1, 3, 5, 1420 | (7 << 32)]
    assert np.uint64(q[1, 2].view(np.uint64)) == np.uint64((1 << 64) - 1)


def test_fault_hooks_only_in_the_test_library():
    """the product library must not read the fault-injection variables (WG_TEST_STEP_FLIP makes
    k_step write wrong tags, WG_RX_TEST_MUTANT restores a racy replay flag). They are compiled only into
    libwgaead_test.so (-DWG_TEST_HOOKS), which the tests needing them load through WG_LIB_PATH."""
    here = os.path.join(ROOT, "wireguard-java_amd")
    prod = open(os.path.join(here, "libwgaead.so"), "rb").read()
    for hook in (b"WG_TEST_STEP_FLIP", b"WG_RX_TEST_SKEW", b"WG_RX_TEST_MUTANT"):
        assert hook not in prod, hook
    test_lib = os.path.join(here, "libwgaead_test.so")
    assert os.path.exists(test_lib), "make -C wireguard-java_amd/csrc test"
    t = open(test_lib, "rb").read()
    for hook in (b"WG_TEST_STEP_FLIP", b"WG_RX_TEST_SKEW", b"WG_RX_TEST_MUTANT"):
        assert hook in t, hook


def test_no_key_codes_declared():
    """WG_ENOKEY / WG_PKT_NOKEY: the per-packet and queue paths refuse a key slot without a key."""
    L = wg()._lib
    src = open(HEADER).read()
    assert f"#define WG_ENOKEY ({L.WG_ENOKEY})" in src
    assert f"#define WG_PKT_NOKEY {L.WG_PKT_NOKEY}u" in src
