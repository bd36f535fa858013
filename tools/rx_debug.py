"""Step-by-step smoke of wg_filter_set / wg_slot_filters_set / wg_rx_check (debug aid)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
from wgtest import wg
W = wg()
dev = torch.device("cuda", 0)
def log(*a):
    print(time.strftime("%H:%M:%S"), *a, flush=True)
e = W.Engine(0, key_slots=64)
log("engine")
e.filter_set(0, [("192.168.1.0", 24), ("2001:db8::", 32)])
log("filter_set")
e.slot_filters_set(0, [0])
log("slot_filters_set")
pt = torch.zeros(256, dtype=torch.uint8, device=dev)
desc = W.pack_desc([0], [0], [0], 40, 0)
d = torch.from_numpy(W.desc_as_int64(desc)).to(dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
log("buffers")
e.rx_check(d, pt, st, 1)
log("rx_check enqueued")
torch.cuda.synchronize()
log("sync", st.cpu().tolist())
e.replay_enable(128)
log("replay_enable")
e.rx_check(d, pt, st, 2)
torch.cuda.synchronize()
log("replay sync", st.cpu().tolist())
e.close()
log("closed")
