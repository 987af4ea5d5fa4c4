import sys, json, os
sys.path.insert(0, os.getcwd())
from kafkabalancer_amd import engine as E, synth
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
cl, cfg, _ = synth.config("c5", scale=scale)
eng = E.Engine(cl, cfg)
for i in range(12):
    ch, err = eng.plan(1)
    st = eng.stats()
    print(json.dumps({"i": i, "err": str(err) if err else None, "ch": ch[0] if ch else None,
                      "contenders": st["contenders"], "exact_folds": st["exact_folds"], "refreshes": st["refreshes"], "halts": st["exact_halts"]}), flush=True)
    if err: break
