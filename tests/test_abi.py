"""The C-ABI boundary: libtsdf_hip.so loads, exports every symbol include/tsdf_hip.h declares, and
fails loudly (no CPU fallback) where no GPU exists.  No compute calls here — CPU suite."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "tsdf_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tsdf_[a-z_]+)\s*\(", txt)))


def dynamic_symbols(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_declares_the_abi():
    fns = header_functions()
    from tsdf_map import _abi
    assert set(fns) == set(_abi.SIGNATURES), "ctypes table out of sync with the header"


def test_hip_library_exports_every_declared_symbol():
    from tsdf_map import HIP_LIB, load_hip_library
    assert os.path.exists(HIP_LIB), "run __graft_entry__.build() first"
    syms = dynamic_symbols(HIP_LIB)
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing
    lib = load_hip_library()
    assert lib.tsdf_abi_version() == 10


def test_hip_library_is_gfx950_code():
    from tsdf_map import HIP_LIB
    out = subprocess.check_output(["strings", HIP_LIB], text=True)
    assert "amdgcn-amd-amdhsa--gfx950" in out


def test_oracle_exports_the_host_subset():
    import oracle
    lib = oracle.load()
    syms = dynamic_symbols(oracle.LIB_PATH)
    for f in header_functions():
        if f in oracle.HOST_ONLY:
            continue
        assert f in syms, f


def test_default_params_roundtrip():
    from tsdf_map import _abi, load_hip_library
    lib = load_hip_library()
    p = _abi.default_params(lib)
    assert p.voxel_size == 0.05 and p.sdf_trunc == 0.15 and p.brick_side == 8
    assert p.space_carving == 0 and np.isinf(p.max_range)
    assert p.walk == _abi.WALK_TWO == 0  # ABI v5: two walks unless the single walk is asked for
    assert p.depth_weight == 1  # ABI v6: Voxblox's 1/z^2 weight, upstream's default
    assert p.voxblox_method == _abi.VB_METHODS["simple"] == 0  # ABI v8
    assert p.sector_input == _abi.SECTOR_INPUTS["fanout"] == 0
    assert p.semantics == _abi.SEM_VDBFUSION_F64  # ABI v8 default
    # ABI v10: SURVEY §8e's contiguous index (column) sectors are the default rule
    assert p.sector_rule == _abi.SECTOR_RULES["index"] == 1
    # the ctypes mirror ends where the C struct ends (ABI v10 appended `sector_rule`)
    assert _abi.TsdfParams._fields_[-1][0] == "sector_rule"


def test_struct_layouts_match_the_header(tmp_path):
    """Every field of tsdf_params / tsdf_stats / tsdf_os_format sits at the same offset, with the
    same size, in the ctypes mirror as in include/tsdf_hip.h compiled by the C compiler."""
    import subprocess
    from tsdf_map import _abi
    structs = {"tsdf_params": _abi.TsdfParams, "tsdf_stats": _abi.TsdfStats,
               "tsdf_os_format": _abi.OsFormat}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "tsdf_hip.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in py._fields_:
            lines.append('printf("%s %s %%zu %%zu\\n", offsetof(%s, %s), sizeof(((%s*)0)->%s));'
                         % (cname, f, cname, f, cname, f))
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    got = {}
    for ln in out:
        parts = ln.split()
        if len(parts) == 3 and parts[1] == "sizeof":
            got[(parts[0], "sizeof")] = int(parts[2])
        elif len(parts) == 4:
            got[(parts[0], parts[1])] = (int(parts[2]), int(parts[3]))
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            fld = getattr(py, f)
            assert got[(cname, f)] == (fld.offset, fld.size), (cname, f)


def test_header_kernel_kinds_match_the_binding():
    """TSDF_K_* of the header name the binding's KERNEL_KINDS (k_<kind>) in order."""
    import re
    from tsdf_map import _abi
    hdr = open(os.path.join(REPO, "include", "tsdf_hip.h")).read()
    kinds = {int(v): k.lower() for k, v in re.findall(r"#define TSDF_K_(\w+) (\d+)", hdr)}
    assert [kinds[i] for i in range(len(kinds))] == list(_abi.KERNEL_KINDS)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is present")
def test_no_gpu_fails_loudly():
    """Without a GPU the product path raises (TSDF_ENODEV); it never falls back to the CPU."""
    from tsdf_map import HipTSDFVolume, TsdfError, _abi
    with pytest.raises(TsdfError) as e:
        HipTSDFVolume(0.05, 0.15)
    assert e.value.code in (_abi.TSDF_ENODEV, _abi.TSDF_EHIP)


def test_invalid_params_rejected_before_device():
    from tsdf_map import _abi, load_hip_library
    lib = load_hip_library()
    for kw in ({"voxel_size": 0.0}, {"sdf_trunc": -1.0}, {"brick_side": 16},
               {"space_carving": 1},  # carving needs a finite max_range
               {"sector_rule": 2}):  # ABI v10: TSDF_SECTOR_RULE_WORLD or _INDEX only
        p = _abi.default_params(lib, **kw)
        ctx = ctypes.c_void_p()
        assert lib.tsdf_create(ctypes.byref(p), ctypes.byref(ctx)) == _abi.TSDF_EINVAL
        assert not ctx.value


def test_backend_switch():
    import tsdf_map
    assert tsdf_map.MAP_BACKEND_IDX == 4
    for idx in range(4):
        with pytest.raises(NotImplementedError):
            tsdf_map.make_backend(idx, voxel_size=0.05, sdf_trunc=0.15)
    with pytest.raises(ValueError):
        tsdf_map.make_backend(9)


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(REPO, "noetic-slam_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h", ".hpp", "Makefile")):
                txt = open(os.path.join(root, f), errors="ignore").read()
                for pat in (r"#\s*include\s*[\"<][^\">]*oracle", r"libtsdf_oracle", r"-ltsdf_oracle",
                            r"^\s*(import|from)\s+oracle", r"oracle/build"):
                    assert not re.search(pat, txt, flags=re.M), (f, pat)


def test_query_dense_takes_int64_bounds():
    """ABI v10: tsdf_query_dense's lo / hi are int64_t[3] in the
    header, in the ctypes table, and in both libraries' behaviour (the oracle, on the CPU): a box
    beyond the int32 range reads the background, and oversized extents are refused."""
    import re
    from tsdf_map import _abi
    hdr = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    proto = re.search(r"int tsdf_query_dense\(([^)]*)\)", hdr).group(1)
    assert "const int64_t lo[3]" in proto and "const int64_t hi[3]" in proto, proto
    args = _abi.SIGNATURES["tsdf_query_dense"][1]
    assert args[1] is ctypes.POINTER(ctypes.c_int64) and args[2] is ctypes.POINTER(ctypes.c_int64)
    import oracle
    v = oracle.OracleTSDFVolume(0.05, 0.15)
    v.integrate(np.array([[2.0, 0.0, 0.0]], np.float32), np.zeros(3))
    big = 1 << 40  # far outside int32 and the index domain (|i| < 2^23)
    s, w = v.query_dense([big, -big, 0], [big + 3, -big + 2, 2])
    assert s.shape == (2, 2, 3) and np.all(s == np.float32(0.15)) and np.all(w == 0)
    # the observed voxels still read back with 64-bit bounds
    s, w = v.query_dense([37, -2, -2], [43, 2, 2])
    assert w.max() > 0
    for lo, hi in (([0, 0, 0], [1 << 31, 1, 1]), ([0, 0, 0], [1 << 14, 1 << 14, 1 << 13]),
                   ([-(1 << 62), 0, 0], [(1 << 62), 1, 1]), ([0, 0, 0], [-1, 1, 1])):
        lo6, hi6 = np.array(lo, np.int64), np.array(hi, np.int64)
        rc = v._lib.tsdf_query_dense(v._ctx, lo6.ctypes.data_as(_abi.L3),
                                     hi6.ctypes.data_as(_abi.L3), None, None)
        assert rc == _abi.TSDF_EINVAL, (lo, hi)
