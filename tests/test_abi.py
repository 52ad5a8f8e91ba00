"""The C-ABI library loads and exports every symbol include/pcn_ipt.h declares (CPU only)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from polycube_amd import ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "pcn_ipt.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pcn_(?:ipt|fw)_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    names = header_functions()
    for must in ("pcn_ipt_create", "pcn_ipt_load_chain", "pcn_ipt_classify", "pcn_ipt_read_counters",
                 "pcn_ipt_set_localip", "pcn_ipt_sync_counters"):
        assert must in names


def test_library_exports_every_header_symbol():
    lib = ffi.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", ffi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (pcn_(?:ipt|fw)_\w+)", out))
    for name in header_functions():
        assert name in exported, name
        assert getattr(lib, name) is not None
    assert set(header_functions()) == set(ffi.SIGNATURES), "ffi.SIGNATURES out of sync with the header"


def test_abi_version():
    assert ffi.lib().pcn_ipt_abi_version() == ffi.ABI_VERSION == 10


def test_classify_fails_loudly_without_device():
    from polycube_amd import Iptables, IptablesError
    ipt = Iptables(device=-1)
    with pytest.raises(IptablesError) as e:
        ipt.classify_ptrs(frames=1, frames_bytes=64, n=1, verdicts=1)
    assert e.value.code == -19  # -ENODEV: no CPU fallback exists
    ipt.close()


def test_chain_program_compiles_without_a_device():
    """The hiprtc chain-program compile (jit.cpp) of classify.hip for config 3's chain."""
    from polycube_amd import Iptables, synth
    ipt = Iptables(device=-1)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in synth.config_rules(3).rules():
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    fw.compile_program()
    assert ipt.jit_info()["programs_ready"] == 1
    ipt.close()


def test_ingest_ring_needs_a_device():
    from polycube_amd import Iptables, IptablesError
    ipt = Iptables(device=-1)
    with pytest.raises(IptablesError) as e:
        ipt.ring(slots=2, slot_frames=16)
    assert e.value.code == -19
    ipt.close()


def test_flow_split_needs_a_device():
    """pcn_ipt_flow_owner / pcn_ipt_flow_split without a device or batch (no GPU
    work is launched).  The rank checks need a device context:
    tests/test_gpu_flow_split.py::test_bad_ranks_are_refused."""
    from polycube_amd import Iptables
    ipt = Iptables(device=-1)
    b = ffi.Batch(1, 64, None, None, 64, 64, None, 1, 0, 0, 0, None, 1, None, None)
    m = C.c_uint64(7)
    lib = ffi.lib()
    assert lib.pcn_ipt_flow_owner(ipt._h, C.byref(b), 2, 1, None) == -19     # -ENODEV, no CPU fallback
    assert lib.pcn_ipt_flow_split(ipt._h, C.byref(b), 2, 0, 1, 1, 1, None, C.byref(m), None) == -19
    assert lib.pcn_ipt_flow_split(ipt._h, None, 2, 0, 1, 1, 1, None, C.byref(m), None) == -22
    ipt.close()


def test_null_context_is_an_error():
    assert ffi.lib().pcn_ipt_chain_flush(None, 0) < 0
    assert b"null" in ffi.lib().pcn_ipt_last_error()
    cfg = ffi.Config(-1, 0, 0, 70000)
    h = C.c_void_p()
    assert ffi.lib().pcn_ipt_create(C.byref(cfg), C.byref(h)) < 0


def test_comm_info_without_a_device():
    """pcn_ipt_comm_get_info with no context: the RCCL that would serve the
    calls (version and library), no device, no gathers."""
    from polycube_amd.iptables import comm_info
    ci = comm_info()
    assert ci["nccl_version"] > 20000 and ci["rccl_version"].count(".") == 2
    assert "rccl" in ci["rccl_path"]
    assert ci["device"] == -1 and ci["gathers_timed"] == 0 and ci["nranks"] == 0


def test_bench_traffic_needs_the_measured_build(tmp_path, monkeypatch):
    """bench.py reports roofline.traffic only for the kernel sources (and batch
    size) the PMC entry was measured on -- the sources embedded in the LOADED
    library, not the files on disk -- and says why not otherwise."""
    import json
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    (tmp_path / "profiles").mkdir()
    h = bench.kernel_src_hash()
    entry = {"frames": 1024, "hbm_bytes_per_launch": 70000, "src_hash": h, "profile": "p"}
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps({"configs": {"config3": entry}}))
    assert bench.load_traffic(3, 0, 1024)[0] == 70000
    assert bench.load_traffic(3, 0, 2048)[0] is None                 # another batch size
    assert bench.load_traffic(5, 1, 1024)[0] is None                 # no entry for config 5 / TC
    monkeypatch.setattr(bench, "kernel_src_hash", lambda: "0123456789abcdef")   # another build loaded
    t, why = bench.load_traffic(3, 0, 1024)
    assert t is None and h in why and "0123456789abcdef" in why


def test_loaded_library_carries_its_sources():
    """The kernel text the library embeds (and compiles chain programs from) is the
    text on disk when the build is fresh, and the build hash covers every source."""
    import bench
    from polycube_amd.iptables import build_sha256
    assert bench.kernel_src_hash() == bench.disk_src_hash()
    for which, rel in ((0, "classify.hip"), (1, "devchain.h"), (3, "image.cpp")):
        with open(os.path.join(bench.ROOT, "polycube_amd", "csrc", rel), "rb") as fh:
            assert ffi.lib().pcn_ipt_embedded_source(which) == fh.read()
    assert ffi.lib().pcn_ipt_embedded_source(4) is None
    assert len(build_sha256()) == 64


def test_program_info_names_the_chain_program():
    """pcn_ipt_get_program_info: the usual launch shape's chain program, compiled on
    the CPU (no device), reports its registers, scratch and deal window."""
    from polycube_amd import Iptables, synth
    ipt = Iptables(device=-1)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in synth.config_rules(2).rules():
        fw.append(**r)
    fw.apply_rules()
    assert fw.program_info()["ready"] == 0
    fw.compile_program()
    pi = fw.program_info()
    assert pi["ready"] == 1 and 0 < pi["vgpr_count"] <= 128 and pi["sgpr_count"] > 0
    assert pi["vgpr_spill_count"] == 0 and pi["deal_window"] == 64 and pi["code_bytes"] > 1000
    assert ipt.chain("INPUT").program_info()["ready"] == 0          # no rules: no program
    ipt.close()
