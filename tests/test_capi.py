"""CPU: libtt2.so loads and exports every entry point include/tt2_capi.h declares,
the ctypes binding covers them, and the ctypes structs match the C layout.
No compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tt2_capi.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"typedef struct.*?\}\s*\w+;", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\*]+\s+\**(tt2_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    from tt2 import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import build_lib
        build_lib.build()
    return _lib


def test_header_parses():
    names = declared_functions()
    assert "tt2_gemm" in names and "tt2_attn_bwd" in names and "tt2_adam_step" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol(lib):
    L = ctypes.CDLL(lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_binding_covers_header(lib):
    assert set(declared_functions()) <= set(lib.SIGNATURES), set(declared_functions()) - set(lib.SIGNATURES)
    lib.load()  # binds argtypes/restype for every entry


def test_struct_sizes_match_c_layout(lib):
    """Compile a tiny host program that prints sizeof/offsetof of the C structs."""
    import subprocess
    import tempfile
    structs = {"tt2_gemm_args": lib.GemmArgs, "tt2_attn_args": lib.AttnArgs, "tt2_ln_args": lib.LnArgs,
               "tt2_bn_args": lib.BnArgs, "tt2_pe_args": lib.PeArgs, "tt2_loss_args": lib.LossArgs,
               "tt2_adam_args": lib.AdamArgs, "tt2_reduce_args": lib.ReduceArgs,
               "tt2_attn_decode_args": lib.AttnDecodeArgs, "tt2_decode_desc": lib.DecodeDesc, "tt2_desc": lib.Desc,
               "tt2_wflip_job": lib.WflipJob, "tt2_ffn_decode_args": lib.FfnDecodeArgs}
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"tt2_capi.h\"\nint main(){\n"
    for name, cls in structs.items():
        last = cls._fields_[-1][0]
        prog += f'printf("{name} %zu %zu\\n", sizeof({name}), offsetof({name}, {last}));\n'
    prog += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "s.c"), os.path.join(d, "s")
        open(src, "w").write(prog)
        r = subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                            "-D__HIP_PLATFORM_AMD__", src, "-o", exe], capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip("host C compiler cannot include hip_runtime_api.h: " + r.stderr[-300:])
        out = subprocess.run([exe], capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        name, size, off = line.split()
        cls = structs[name]
        last = cls._fields_[-1][0]
        assert ctypes.sizeof(cls) == int(size), name
        assert getattr(cls, last).offset == int(off), name


def test_no_cpu_fallback(lib):
    """The product path raises without a GPU instead of computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(lib.TT2Error):
        lib.lib()


def test_block_sizes_without_gpu(lib):
    """The block-level size queries are host-only (the dry pass of each block, no device
    call): positive, growing with the batch, 0 for an invalid descriptor."""
    import ctypes as C
    L = lib.load()

    def desc(batch, **kw):
        d = lib.Desc()
        d.batch, d.tq, d.tk, d.d_model, d.n_heads, d.d_ffn = batch, 800, 128, 512, 8, 2048
        d.c_in, d.c_out, d.kernel, d.dtype, d.n_mels, d.heads_ld = 512, 512, 5, lib.DT_BF16, 80, 96
        for k, v in kw.items():
            setattr(d, k, v)
        return d

    for fn in ("tt2_attn_block_saved_size", "tt2_attn_block_workspace_size", "tt2_ffn_saved_size",
               "tt2_ffn_workspace_size", "tt2_linear_workspace_size", "tt2_add_ln_saved_size",
               "tt2_add_ln_workspace_size", "tt2_conv1d_bn_act_saved_size", "tt2_conv1d_bn_act_workspace_size",
               "tt2_heads_workspace_size", "tt2_loss_block_workspace_size"):
        f = getattr(L, fn)
        small, big = f(C.byref(desc(2))), f(C.byref(desc(16)))
        assert 0 < small <= big, fn
    assert L.tt2_attn_block_saved_size(C.byref(desc(2, cross=1))) > 0
    assert L.tt2_attn_block_saved_size(C.byref(desc(2, d_model=384))) == 0
    assert L.tt2_conv1d_bn_act_workspace_size(C.byref(desc(2, kernel=4))) == 0
