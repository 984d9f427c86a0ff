"""The C-ABI library loads and exports every entry point include/nbx.h declares
(CPU-only: no compute call touches a device)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "nbx.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(nbx_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def L():
    import nbody_amd._lib as lib
    if not os.path.exists(lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return lib.lib()


def test_header_declares_the_path():
    syms = declared_symbols()
    for s in ["nbx_fc_edge_index", "nbx_knn_edge_index", "nbx_gravity_acceleration", "nbx_gravity_sample",
              "nbx_segnn_forward", "nbx_segnn_rollout", "nbx_segnn_workspace_bytes", "nbx_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol(L):
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version_and_host_only_calls(L):
    import nbody_amd._lib as lib
    assert L.nbx_abi_version() == lib.ABI_VERSION
    n = lib.c_sz()
    assert L.nbx_segnn_workspace_bytes(1024, 5, 96, ctypes.byref(n)) == 0
    assert n.value > 100 * 2 ** 20
    # argument validation happens before any device call and reports through nbx_last_error
    assert L.nbx_fc_edge_index(-1, 5, None, None) == 1
    assert b"bad sizes" in L.nbx_last_error()
    assert L.nbx_knn_edge_index(None, 0, 1, 5, 5, None, None) == 1
    assert b"more neighbors" in L.nbx_last_error()


def _struct_fields(name):
    """(field names, pointer count) of `typedef struct name {...} name;` in include/nbx.h."""
    import re
    txt = open(os.path.join(ROOT, "include", "nbx.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), txt, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(\w+)\s*(?:\[[^\]]*\])?;", body)
    ptrs = len(re.findall(r"\*\s*\w+;", body))
    return fields, ptrs


def test_struct_layout_matches_header():
    """ctypes mirror of nbx_segnn_weights has the C layout: same fields, same order,
    pointer-aligned sizes."""
    import nbody_amd._lib as lib
    lf, layer_ptrs = _struct_fields("nbx_segnn_layer")
    assert [f for f, _ in lib.SegnnLayer._fields_] == lf
    layer_bytes = layer_ptrs * 8 + 4 * 4   # + the four fp16x2 descale factors (ABI 15)
    assert ctypes.sizeof(lib.SegnnLayer) == layer_bytes
    wf, w_ptrs = _struct_fields("nbx_segnn_weights")
    assert [f for f, _ in lib.SegnnWeights._fields_] == wf
    head = 3 * 4 + 2 * 4   # mul, num_layers, training, bn_eps, bn_momentum
    head = (head + 7) // 8 * 8
    # bn_allreduce (function pointer), bn_global_batch (int64), deterministic + reserved0,
    # pp1_h2_descale + reserved1
    extra = 8 + 8 + 8 + 8
    assert ctypes.sizeof(lib.SegnnWeights) == head + w_ptrs * 8 + extra + lib.MAX_LAYERS * layer_bytes


def test_struct_offsets_match_the_c_compiler(tmp_path):
    """Every field offset and struct size of the ctypes mirrors equals what gcc computes
    from include/nbx.h (the header is plain C)."""
    import shutil
    import subprocess

    import nbody_amd._lib as lib
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    structs = {"nbx_segnn_layer": lib.SegnnLayer, "nbx_segnn_weights": lib.SegnnWeights,
               "nbx_egnn_layer": lib.EgnnLayer, "nbx_egnn_head": lib.EgnnHead, "nbx_egnn_weights": lib.EgnnWeights,
               "nbx_ponita_layer": lib.PonitaLayer, "nbx_ponita_weights": lib.PonitaWeights,
               "nbx_eqv2_radial": lib.Eqv2Radial, "nbx_eqv2_attn": lib.Eqv2Attn, "nbx_eqv2_block": lib.Eqv2Block,
               "nbx_eqv2_weights": lib.Eqv2Weights}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "nbx.h"', "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, cls in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_product_fails_loudly_without_device():
    """No CPU fallback: the HIP-only ops raise on CPU tensors."""
    import torch

    import nbody_amd._lib as lib
    with pytest.raises(lib.NbxError):
        lib.dev_ptr(torch.zeros(3))


def test_isa_scan_flags_the_measured_hazard_only(tmp_path):
    """The gfx950 MFMA SrcA hazard check build.py runs (nbody_amd/isa_scan.py): a load in the
    slot right after a v_mfma_f32_16x16x32_bf16 that writes its SrcA is flagged; one wait state
    in between, a SrcB overwrite, or another MFMA shape is not (tools/hazard/mfma_war.hip)."""
    from nbody_amd.isa_scan import scan
    body = """kern:
\tv_mfma_f32_16x16x32_bf16 v[8:11], v[0:3], v[4:7], v[8:11]
\tds_read_b128 v[0:3], v20
\tv_mfma_f32_16x16x32_bf16 v[8:11], v[0:3], v[4:7], v[8:11]
\ts_nop 0
\tds_read_b128 v[0:3], v20
\tv_mfma_f32_16x16x32_bf16 v[8:11], v[0:3], v[4:7], v[8:11]
\tbuffer_load_dwordx4 v[4:7], v21, s[0:3], 0 offen
\tv_mfma_f32_32x32x16_bf16 v[8:23], v[0:3], v[4:7], v[8:23]
\tds_read_b128 v[0:3], v20
\tv_mfma_f32_16x16x32_bf16 v[8:11], v[0:3], v[4:7], v[8:11]
\tbuffer_load_dwordx4 v[2:5], v21, s[0:3], 0 offen
"""
    p = tmp_path / "k.s"
    p.write_text(body)
    hits = scan(str(p), 1, rule=True)
    assert [(h[2], h[6]) for h in hits] == [(3, "SrcA"), (12, "SrcA")]
    assert len(scan(str(p), 4)) > len(hits)        # the broad scan lists the safe pairs too


def test_built_kernels_free_of_the_mfma_srca_hazard():
    import glob

    from nbody_amd.build import ISA_DIR
    from nbody_amd.isa_scan import scan
    files = glob.glob(os.path.join(ISA_DIR, "*.s"))
    if not files:
        pytest.skip("no device assembly (library not built here)")
    assert [h for f in files for h in scan(f, 1, rule=True)] == []
