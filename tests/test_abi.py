"""CPU: the C-ABI libraries load and export every symbol the headers declare;
the introspection entry points work without a GPU. No compute calls."""
import ctypes
import os
import re

import pytest

import xucg_amd
from xucg_amd import _lib
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ucg_builtin_\w+)\s*\(", text)))


def test_dev_library_exports_every_declared_symbol():
    names = declared("ucg_builtin_dev.h")
    assert len(names) >= 20
    lib = ctypes.CDLL(_lib.DEV_LIB)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding covers exactly the declared surface
    assert sorted(_lib.DEV_API) == names


def test_host_library_exports_every_declared_symbol():
    names = sorted(set(declared("ucg_builtin_combine.h")) | set(declared("ucg_builtin_ops.h")) |
                   set(declared("ucg_builtin_component.h")))
    assert len(names) >= 10
    lib = ctypes.CDLL(_lib.HOST_LIB)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from xucg_amd import host_api
    assert sorted(host_api.HOST_API) == names


def test_support_table_matches_oracle():
    for dt in range(len(O.DTYPES)):
        assert xucg_amd.dtype_size(dt) == O.lib().ucg_oracle_dtype_size(dt)
        assert _lib.dev().ucg_builtin_dev_dtype_size(dt) == xucg_amd.dtype_size(dt)
        for op in range(len(O.OPS)):
            assert xucg_amd.is_supported(dt, op) == O.is_supported(dt, op)
    assert not xucg_amd.is_supported(99, 0)
    assert not xucg_amd.is_supported(0, 99)


def test_version_and_errors_without_gpu():
    assert b"gfx950" in _lib.dev().ucg_builtin_dev_version()
    if xucg_amd.device_count() > 0:
        pytest.skip("a GPU is visible; the no-device path is not reachable")
    with pytest.raises(xucg_amd.UcsError) as e:
        xucg_amd.DevContext(device=0)
    assert e.value.status == xucg_amd.UCS_ERR_NO_DEVICE
    # NULL context is rejected, not dereferenced
    L = _lib.dev()
    assert L.ucg_builtin_dev_reduce(None, 0, 10, None, None, 4) == _lib.UCS_ERR_INVALID_PARAM
    assert L.ucg_builtin_dev_sync(None) == _lib.UCS_ERR_INVALID_PARAM
    assert L.ucg_builtin_dev_stage_end(None) == _lib.UCS_ERR_INVALID_PARAM


def test_host_library_exports_the_plan_component():
    """The drop-in boundary: the global ucg_builtin_component of type
    ucg_plan_component_t (api/ucg_plan_component.h:141-188, defined as
    builtin/builtin.c:1007-1016 defines it), already registered in
    ucg_plan_components_list by its load-time constructor."""
    lib = ctypes.CDLL(_lib.HOST_LIB)
    comp = ctypes.c_char.in_dll(lib, "ucg_builtin_component")
    name = ctypes.string_at(ctypes.addressof(comp), 16).split(b"\0")[0]
    assert name == b"builtin"
    head = (ctypes.c_void_p * 2).in_dll(lib, "ucg_plan_components_list")
    assert head[1] != ctypes.addressof(head), "component not in ucg_plan_components_list"


def _kernel_metadata(obj):
    """(name, vgpr_count, group_segment_fixed_size) of every gfx950 kernel in
    a hipcc object: the .hip_fatbin section, unbundled, its AMDGPU notes"""
    import re
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                        os.path.join(d, "junk")], check=True, capture_output=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                        f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out = []
    for block in notes.split("\n  - .agpr_count:")[1:]:
        name = re.search(r"\n    \.name:\s+(\S+)", block).group(1)
        vgpr = int(re.search(r"\n    \.vgpr_count:\s+(\d+)", block).group(1))
        lds = int(re.search(r"\n    \.group_segment_fixed_size:\s+(\d+)", block).group(1))
        out.append((name, vgpr, lds))
    return out


def test_kernel_resources():
    """Round 4: no product kernel allocates LDS, and the
    occupancy cap of the multi-operand kernels is their register allocation:
    every capped k_reduce_multi / k_reduce_tree (CAP template argument 1)
    holds at least 168 VGPRs - at most 3 waves per SIMD, 12 per CU (a few
    byte-wide kernels need more registers of their own) - while the uncapped
    fp32 / fp64 SUM forms fit more. Read from the built objects' code-object
    metadata."""
    import glob
    import re
    objs = sorted(glob.glob(os.path.join(ROOT, "xucg_amd", "csrc", "_obj", "dev_inst_*.o")) +
                  glob.glob(os.path.join(ROOT, "xucg_amd", "csrc", "_obj", "dev_combine.o")))
    if not objs or not os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler"):
        pytest.skip("the device objects are not built here")
    capped = uncapped = 0
    for obj in objs:
        for name, vgpr, lds in _kernel_metadata(obj):
            assert lds == 0, (obj, name, lds)
            # template arguments T, OP, N, XM, CAP, PF, PFM, PFD, PFO: CAP
            # is the fourth integer (round 5 added the prefetch arguments,
            # round 6 the prefetch order)
            m = re.match(r"_ZN6ucgdev1[34]k_reduce_(multi|tree)I([fd])?", name)
            ints = re.findall(r"Li(\d+)E", name)
            if m and len(ints) == 8:
                if ints[3] == "1":
                    capped += 1
                    assert vgpr >= 168, (name, vgpr)
                elif m.group(2):
                    uncapped += 1
                    assert vgpr < 168, (name, vgpr)
    assert capped > 0 and uncapped > 0, (capped, uncapped)


def test_code_object_hash_keys_kernel_counters(tmp_path, monkeypatch):
    """PMC traffic is keyed to the device code (.hip_fatbin of
    libucg_builtin_dev.so), not the whole library: the hash is found, is
    stable, is not the file's hash, and bench.py's pmc_traffic calls a
    summary of the same code fresh even when the library hash differs (a
    host-only edit), and stale when the code differs."""
    import hashlib
    import json
    import sys
    code = _lib.code_object_sha16()
    assert code and len(code) == 16 and code == _lib.code_object_sha16()
    whole = hashlib.sha256(open(_lib.DEV_LIB, "rb").read()).hexdigest()[:16]
    assert code != whole
    assert _lib.code_object_sha16(_lib.HOST_LIB) is None     # no device code there
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"hbm_bytes_per_launch": 811463936, "source": "x", "lib_sha16": "0" * 16,
             "code_sha16": code}
    (prof / "pmc_traffic.json").write_text(json.dumps({"67108864": entry}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src = bench.pmc_traffic(1 << 26)
    assert traffic == 811463936 and src["stale"] is False
    assert src["keyed_by"].startswith("code object")
    entry["code_sha16"] = "f" * 16
    (prof / "pmc_traffic.json").write_text(json.dumps({"67108864": entry}))
    assert bench.pmc_traffic(1 << 26)[1]["stale"] is True
