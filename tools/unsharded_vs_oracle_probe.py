import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from kafkabalancer_amd import engine as E, synth
from helpers import default_cfg, oracle_plan, key
cl = synth.make_cluster(2500, 40, 3, "zipf", nsets=8, set_size=24, seed=5, with_names=True)
cfg = default_cfg(allow_leader=True, min_unbalance=0.0)
eng = E.Engine(cl, cfg)
ch, err = eng.plan(24)
pl = synth.to_plist(cl)
och, oerr, opl = oracle_plan(pl, cfg, 24)
a = [key(c) for c in ch]; b = [key(c) for c in och]
print("unsharded == oracle:", a == b, len(a), len(b), err, oerr)
for i, (x, y) in enumerate(zip(a, b)):
    if x != y: print("first diff", i, x, y); break
print("state equal:", eng.state() == opl.state())
