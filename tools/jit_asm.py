"""Assembly + resource usage of a chain program (inspection tool, CPU only).

Builds config N's FORWARD chain on a device-less context, rebuilds the same
pcn_jit_spec.h that jit.cpp generates for the usual launch shape, compiles
classify.hip with hipcc -DPCN_JIT -S and prints the kernel's register/LDS/
occupancy remarks plus an instruction histogram of its main loop.

  python tools/jit_asm.py [--cfg 3] [--defs "-DPCN_ABLATE=2"] [--out /tmp/jit.s]
"""
import argparse
import collections
import ctypes as C
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def layout_words():
    src = open(os.path.join(ROOT, "polycube_amd", "csrc", "devchain.h")).read()
    body = src[src.index("struct TableLayout"):src.index("};", src.index("struct TableLayout"))]
    n = 0
    for line in body.splitlines()[1:]:
        line = line.split("//")[0].strip()
        if not line.startswith("uint32_t"):
            continue
        for part in line[len("uint32_t"):].rstrip(";").split(","):
            m = re.search(r"\[(\d+)\]", part)
            n += int(m.group(1)) if m else 1
    return n


def spec_for(cfg, imix=False, inputs=0):
    from polycube_amd import Iptables, ffi, synth
    rs = synth.config_rules(cfg)
    ipt = Iptables(device=-1, max_rules=16384, max_counted_rules=10000)
    ipt.interactive = False
    fw = ipt.chain("FORWARD")
    for r in rs.rules():
        fw.append(**r)
    fw.default = "DROP"
    fw.apply_rules()
    desc = (C.c_uint32 * 256)()
    ffi.lib().pcn_ipt_chain_get_image(ipt._h, 1, None, 0, desc, 256)
    nl = layout_words()
    lay = [desc[i] for i in range(nl)]
    nrw, nsw, present, all_cls = (desc[nl + i] for i in range(4))
    info = fw.info()
    ncounted = min(info["nrules"], 10000 if cfg == 5 else 8000)
    lds_bins = 3 if ncounted <= 2048 else -1
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from image_model import LAYOUT
    ns = lay[LAYOUT.index("nslots")]
    vals = ", ".join(f"{x}u" for x in lay)
    # --imix: the offsets/lens launch shape with the staged prefix [0, pbase) (config 5's)
    limit = lay[LAYOUT.index("pbase")] if imix else lay[0]
    return (f"#pragma once\n#define PCN_JIT_FIXED {'false' if imix else 'true'}\n#define PCN_JIT_LDS true\n#define PCN_JIT_CH 1\n"
            f"#define PCN_JIT_NS {ns}\n#define PCN_JIT_INPUTS {inputs}\n#define PCN_JIT_CHAIN {{{vals}, nullptr, nullptr, {info['nrules']}u, {nrw}u, "
            f"{nsw}u, {present}u, {info['nvec']}u, {all_cls}u, {ncounted}u, 10000u, 0, 0u, {limit}u, {lds_bins}}}\n"
            + ("#ifndef PCN_DEAL2\n#define PCN_DEAL2 2\n#endif\n" if nsw >= 2 else ""))   # as jit.cpp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--defs", default="")
    ap.add_argument("--out", default="/tmp/pcn_jit.s")
    ap.add_argument("--imix", action="store_true", help="offsets/lens launch shape (FIXED false, prefix staged)")
    ap.add_argument("--inputs", type=int, default=0, help="PCN_JIT_INPUTS (8: stale ports, 16: Horus table)")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp()
    with open(os.path.join(tmp, "pcn_jit_spec.h"), "w") as fh:
        fh.write(spec_for(a.cfg, a.imix, a.inputs | (96 if a.imix else 0)))   # + offsets and lens arrays
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", f"-I{ROOT}/include", f"-I{ROOT}/polycube_amd/csrc",
           f"-I{tmp}", "-DPCN_JIT", *a.defs.split(), "--offload-arch=gfx950", "-x", "hip", "--cuda-device-only",
           "-S", f"{ROOT}/polycube_amd/csrc/classify.hip", "-o", a.out, "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*) \[-Rpass", line)
        if m and any(k in m.group(1) for k in ("VGPRs", "SGPRs", "Scratch", "Occupancy", "LDS")):
            print(m.group(1))
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(1)
    ins = [ln.split()[0] for ln in open(a.out) if re.match(r"\s+(v_|s_|ds_|global_|buffer_)", ln)]
    hist = collections.Counter(ins)
    print(f"{len(ins)} instructions;", ", ".join(f"{k} {v}" for k, v in hist.most_common(25)))


if __name__ == "__main__":
    main()
