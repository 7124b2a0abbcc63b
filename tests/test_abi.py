"""CPU checks of the C-ABI boundary (include/kplace.h): the library loads,
exports every declared symbol, documents its defaults, and the host-side
helpers behave; no kernel runs here (no GPU in this container)."""
import ctypes as C
import os
import re

import pytest

from kplace import _abi

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                   "kplace.h")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_abi.LIB_PATH):
        import __graft_entry__  # noqa: F401  (tests run from the repo root)
        __graft_entry__.build()
    return _abi.load_library()


def declared_symbols():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(kp_\w+)\s*\(", src, re.M)))


def test_header_and_binding_agree():
    assert sorted(_abi.EXPORTED) == declared_symbols()


def test_exports_every_declared_symbol(lib):
    for sym in declared_symbols():
        assert hasattr(lib, sym), sym


def test_struct_layouts_match_header(tmp_path):
    """Field offsets of every ctypes mirror equal the C compiler's."""
    import subprocess
    structs = {"kp_snapshot": _abi.Snapshot, "kp_params": _abi.Params, "kp_result": _abi.Result,
               "kp_config": _abi.Config, "kp_timing": _abi.Timing,
               "kp_preemption": _abi.Preemption}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                 check=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"


def test_abi_version(lib):
    assert lib.kp_abi_version() == _abi.KP_ABI_VERSION


def test_params_default_matches_documentation(lib):
    p = _abi.Params()
    lib.kp_params_default(C.byref(p))
    assert _abi.params_dict(p) == _abi.params_dict(_abi.default_params())


def test_strerror(lib):
    for code in (0, -1, -2, -3, -4, -5, -6, -99):
        assert lib.kp_strerror(code)


@pytest.mark.parametrize("s,want", [
    ("2Gi", 2048), ("24Gi", 24576), ("512Mi", 512), ("0Mi", 0), ("", 0),
    ("1Gi", 1024), ("288Gi", 294912),
])
def test_parse_gpu_memory_ok(lib, s, want):
    v = C.c_int64(-1)
    assert lib.kp_parse_gpu_memory(s.encode(), C.byref(v)) == 0
    assert v.value == want


@pytest.mark.parametrize("s", ["2G", "Gi", "2gi", "-2Gi", "2.5Gi", " 2Gi", "2Gi ", "2Ki",
                               "99999999999999999999Gi", "9007199254740993Gi"])
def test_parse_gpu_memory_rejects(lib, s):
    v = C.c_int64(-1)
    assert lib.kp_parse_gpu_memory(s.encode(), C.byref(v)) == _abi.KP_EINVAL


def test_create_without_gpu_fails_loudly(lib):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    h = C.c_void_p()
    assert lib.kp_create(C.byref(h), None) == _abi.KP_ENODEV
    assert not h.value


def test_null_args_rejected(lib):
    assert lib.kp_create(None, None) == _abi.KP_EINVAL
    assert lib.kp_solve(None, None, None) == _abi.KP_EINVAL
    assert lib.kp_place(None, None, None, None) == _abi.KP_EINVAL
    assert lib.kp_dist_unique_id(None) == _abi.KP_EINVAL
