"""Debug: config-1 parity on the GPU, repeated, with mismatch positions."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
import os
from polycube_amd import ffi
if os.environ.get("PCN_LIB"): ffi.LIB_PATH = os.environ["PCN_LIB"]
from polycube_amd import Iptables, synth
from oracle.ffi import Oracle
from image_model import ImageModel, model_classify
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = 1 << 16
rs = synth.config_rules(cfg); rules = rs.rules()
ipt = Iptables(device=0); ipt.interactive = False
fw = ipt.chain("FORWARD")
for r in rules: fw.append(**r)
fw.default = "DROP"; fw.apply_rules()
print(fw.info())
o = Oracle(); o.set_chain(1, rules, "DROP")
fr = synth.config_frames(cfg, n, rs).reshape(-1)
v, r = o.classify(fr, n=n)
t = torch.from_numpy(fr).cuda()
for rep in range(4):
    vg, rg = ipt.classify(t, n=n); torch.cuda.synchronize()
    rg = rg.cpu().numpy()
    bad = np.nonzero(rg != r)[0]
    print("rep", rep, "mismatch", bad.size, bad[:12], r[bad[:12]], rg[bad[:12]])
    if bad.size:
        lanes = bad % 64; waves = bad // 64
        print("   waves", np.unique(waves)[:20], "lanes", np.unique(lanes)[:40])
rr = rg
print("desc-check markers:", [(k, int(v)) for k, v in enumerate(rr[:512]) if v <= -1000][:20])
