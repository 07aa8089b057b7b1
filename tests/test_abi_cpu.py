"""CPU-side checks of the C-ABI boundary: libmtts.so loads, exports every
symbol include/mtts.h declares, and the ctypes struct layouts match the C
compiler's (sizeof + offsetof, compiled with gcc from the header)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mtts.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(mtts_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from mtts import _lib
    lib = _lib.lib()
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), f"libmtts.so does not export {n}"
    assert set(names) == set(_lib.exported_symbols())
    assert lib.mtts_abi_version() == _lib.ABI_VERSION


STRUCTS = {
    "MttsScanFwdArgs": "ScanFwdArgs", "MttsScanBwdArgs": "ScanBwdArgs", "MttsConvFwdArgs": "ConvFwdArgs",
    "MttsConvBwdArgs": "ConvBwdArgs", "MttsConvUpdateArgs": "ConvUpdateArgs",
    "MttsStateUpdateArgs": "StateUpdateArgs", "MttsLNArgs": "LNArgs", "MttsLNBwdArgs": "LNBwdArgs",
    "MttsAttnFwdArgs": "AttnFwdArgs", "MttsAttnBwdArgs": "AttnBwdArgs", "MttsCastDesc": "CastDesc",
    "MttsAdamTensor": "AdamTensor", "MttsRowsArgs": "RowsArgs", "MttsGemmArgs": "GemmArgs", "MttsSkinnyArgs": "SkinnyArgs",
    "MttsDropoutArgs": "DropoutArgs", "MttsConvGemmArgs": "ConvGemmArgs",
}


def test_ctypes_layout_matches_c_header():
    from mtts import _lib
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, pyname in STRUCTS.items():
        lines.append(f'printf("{pyname} size %zu\\n", sizeof({cname}));')
        for fname, _ in getattr(_lib, pyname)._fields_:
            lines.append(f'printf("{pyname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c11", c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    for line in out.strip().splitlines():
        py, field, val = line.split()
        cls = getattr(_lib, py)
        got = ctypes.sizeof(cls) if field == "size" else getattr(cls, field).offset
        assert got == int(val), f"{py}.{field}: ctypes {got} != C {val}"


def test_ops_refuse_cpu_tensors():
    import torch
    from mtts import ops
    u = torch.zeros(1, 4, 8)
    with pytest.raises(RuntimeError, match="no CPU path"):
        ops.scan_fwd(u, u, torch.zeros(8, 16), torch.zeros(1, 4, 16), torch.zeros(1, 4, 16))


def test_drop_in_modules_keep_reference_state_dict_keys(golden):
    import mamba_decoder
    import style_cross_attention as sca
    g = golden("decoder.npz")
    m = mamba_decoder.MambaTTSDecoder(vocab_size_audio=10, d_model=64, n_layers=2, n_heads=4, d_ff=128,
                                      d_style=16, max_len=256)
    ref_keys = {k[3:] for k in g if k.startswith("sd/")}
    assert set(m.state_dict().keys()) == ref_keys
    for k, v in m.state_dict().items():
        assert tuple(v.shape) == g["sd/" + k].shape, k
    s = golden("style.npz")
    p = sca.StyleConditioningPipeline(d_style=16, d_model=64, num_heads=4)
    assert set(p.state_dict().keys()) == {k[3:] for k in s if k.startswith("sd/")}
