"""C-ABI boundary checks that need no GPU: the library loads, exports every symbol include/hlmc.h
declares, validates arguments without touching the device, and describes parameter layouts that
match the drop-in nn.Modules."""
import ctypes as C
import re

import pytest
import torch

import hlmc_amd
from hlmc_amd import _lib as L


def header_symbols():
    src = open("include/hlmc.h").read()
    return sorted(set(re.findall(r"\b(hlmc_[A-Za-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = L.lib()
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(header_symbols()) == set(L.exported_symbols()), "ctypes table out of sync with the header"
    assert lib.hlmc_version() == 1


def test_library_resolves_every_symbol_at_load():
    """RTLD_NOW binding: an internal function declared but never defined fails here, not in a GPU call."""
    import os
    C.CDLL(L.LIB_PATH, mode=os.RTLD_NOW | os.RTLD_LOCAL)


def test_bad_arguments_return_einval_with_message():
    lib = L.lib()
    h = C.c_void_p()
    assert lib.hlmc_net_create(7, L.i64_array([1]), 1, 0, C.byref(h)) == -1
    assert b"unknown net kind" in lib.hlmc_last_error()
    assert lib.hlmc_net_create(0, L.i64_array([128, 768, 100, 128]), 4, 0, C.byref(h)) == -1
    assert b"multiples of 64" in lib.hlmc_last_error()
    assert lib.hlmc_mel_plan_create(22050, 1024, 512, 128, 0.0, 0.0, C.byref(h)) == -1
    with pytest.raises(L.HLMCError):
        L.check(lib.hlmc_net_create(0, L.i64_array([128]), 1, 0, C.byref(h)))


@pytest.mark.parametrize("make", [
    lambda: hlmc_amd.HybridVAE(128, 768, (128, 128)),
    lambda: hlmc_amd.HybridVAE(128, 384, (128, 128), audio_only=True),
    lambda: hlmc_amd.HybridVAE(),
    lambda: hlmc_amd.ConditionalVAE(64, 768, 10, (128, 128)),
    lambda: hlmc_amd.ConditionalVAE(),
    lambda: hlmc_amd.VAE(370, [128, 64, 32], 32),
])
def test_native_layout_matches_module(make):
    m = make()
    for dt in (0, 1):
        net = hlmc_amd.models.NativeNet(m._kind, m._native_cfg(), dt)
        net.check_module(m)
        assert net.workspace_bytes(4) > 0


def test_state_dict_identical_to_oracle():
    from oracle import models_oracle as OM
    torch.manual_seed(42)
    a = OM.HybridVAE(128, 768, (128, 128))
    torch.manual_seed(42)
    b = hlmc_amd.HybridVAE(128, 768, (128, 128))
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert ka == kb and torch.equal(va, vb)


def test_modules_refuse_cpu_execution():
    m = hlmc_amd.HybridVAE(128, 768, (128, 128))
    with pytest.raises(L.HLMCError):
        m(torch.zeros(2, 1, 128, 128), torch.zeros(2, 768))
