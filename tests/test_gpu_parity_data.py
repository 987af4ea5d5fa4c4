"""Random small partition lists shared by the parity tests and the golden generator."""


def random_plist(rng, P, B, weights, sets, nrvar, ncons=False):
    parts = []
    for i in range(P):
        rf = rng.randint(1, min(3, B))
        reps = rng.sample(range(1, B + 1), rf)
        p = {"topic": "t%d" % (i % 7), "partition": i, "replicas": reps}
        if weights == "int":
            p["weight"] = float(rng.randint(1, 5))
        elif weights == "zipf":
            p["weight"] = rng.uniform(1, 1000) ** -1.1
        if sets == "some" and rng.random() < 0.5:
            p["brokers"] = sorted(rng.sample(range(1, B + 3), rng.randint(1, B + 2)))
        elif sets == "all":
            p["brokers"] = sorted(rng.sample(range(1, B + 1), rng.randint(max(1, B // 2), B)))
        if nrvar and rng.random() < 0.1:
            p["num_replicas"] = max(1, rf + rng.choice([-1, 1]))
        if ncons and rng.random() < 0.3:
            p["num_consumers"] = rng.randint(0, 3)
        parts.append(p)
    if weights in ("int", "zipf") and parts and "weight" not in parts[0]:
        parts[0]["weight"] = 1.0
    return {"version": 1, "partitions": parts}
