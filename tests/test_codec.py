"""Codec fast path (kafkabalancer_amd/host/codecs.cpp, §8(f1)): the one-pass JSON
decoder must give exactly what the DOM parser + decoder gives (result bytes or
error text), and the encoder must write the reference's bytes (codecs.go:15-27,
84-93; the oracle's writer is the pin).  CPU only: no engine is created."""
import json
import random

import pytest

from kafkabalancer_amd import cli, synth
from oracle import oracle as O

from helpers import golden


def same_as_dom(data):
    """The CLI's path (fast, DOM fallback) and the DOM path agree; returns the
    one-pass decoder's own verdict (0 = it decoded the input itself)."""
    rc0, o0, *_ = cli.codec_roundtrip(data, cli.CODEC_DEFAULT)
    rc1, o1, *_ = cli.codec_roundtrip(data, cli.CODEC_DOM)
    assert (rc0, o0) == (rc1, o1), (data[:200], o0[:200], o1[:200])
    # (the one-pass decoder alone skips the version / empty checks that follow it)
    rc2, o2, *_ = cli.codec_roundtrip(data, cli.CODEC_FAST)
    if rc2 == 0 and rc1 == 0:
        assert o1 == o2
    return rc2


def synthetic(n=2000, seed=5):
    cl = synth.make_cluster(n, 100, 3, "zipf", nsets=16, set_size=24, seed=seed, with_names=True)
    return synth.to_plist(cl)


def test_golden_fixture():
    assert same_as_dom(json.dumps(golden("test.json")).encode()) == 0
    with open("tests/golden/test.json", "rb") as f:
        assert same_as_dom(f.read()) == 0


@pytest.mark.parametrize("threads", ["1", "3"])
def test_synthetic_matches_oracle_writer(threads, monkeypatch):
    monkeypatch.setenv("KB_CODEC_THREADS", threads)          # the encoder's slice split
    pl = synthetic(10000)
    data = json.dumps(pl).encode()
    rc, got, tp, te, n = cli.codec_roundtrip(data)
    assert rc == 0 and n == 10000
    code, want, err = O.run_plan(O.OraclePL(pl), O.default_cfg(), max_reassign=0, full_output=True)
    assert code == 0, err
    assert got == want
    assert same_as_dom(data) == 0


EDGE = [
    b'{"version":1,"partitions":[]}',
    b'{"version":1,"partitions":null}',
    b'{"version":1}',
    b'{}',
    b'{"version":1,"partitions":[null,{"topic":"a","partition":3,"replicas":[1,2]}]}',
    b' \n\t{"Version" : 1 , "PARTITIONS":[{"Topic":"x","Partition":-0,"Replicas":null,"Weight":null}]} trailing',
    b'{"version":1,"partitions":[{"topic":"a","replicas":[1],"replicas":[2,3],"weight":1.5e-300,"weight":2}]}',
    b'{"version":1,"partitions":[{"topic":"a","partitions":1}],"partitions":[{"topic":"b","partition":9223372036854775807}]}',
    b'{"version":1,"partitions":[{"topic":"b","partition":-9223372036854775808,"num_consumers":7,"num_replicas":3}]}',
    b'{"version":1,"partitions":[{"topic":"b","partition":9223372036854775808}]}',
    b'{"version":1,"partitions":[{"topic":"b","partition":1.0}]}',
    b'{"version":1,"partitions":[{"topic":"b","partition":1e3}]}',
    b'{"version":1,"partitions":[{"topic":"b","weight":1e400}]}',
    b'{"version":1,"partitions":[{"topic":"b","weight":4.9e-325}]}',
    b'{"version":1,"partitions":[{"topic":"b\\u00e9\\n<&>","partition":1,"replicas":[1]}]}',
    b'{"version":1,"partitions":[{"topic":"\xc3\xa9\xff raw","partition":1,"replicas":[1]}]}',
    b'{"version":1,"partitions":[{"topic":"b","extra":{"x":[1,2,{"y":null}]},"replicas":[1]}]}',
    b'{"version":2,"partitions":[{"topic":"b","replicas":[1]}]}',
    b'{"version":1,"partitions":[{"topic":"b","replicas":[1,]}]}',
    b'{"version":1,"partitions":[{"topic":"b","replicas":[01]}]}',
    b'{"version":1,"partitions":[{"topic":"b","replicas":["1"]}]}',
    b'{"version":1,"partitions":{"topic":"b"}}',
    b'[1,2]',
    b'',
    b'   ',
    b'{"version":1,"partitions":[{"topic":"b","weight":-0.0,"replicas":[1]}',
    b'{"version":1,"partitions":[{"topic":"b","weight":1e21,"num_replicas":2,"brokers":[],"replicas":[4,5]}]}',
    b'{"version":1,"partitions":[{"topic":"b","weight":0.000001,"brokers":[3,1],"replicas":[4,5]}]}',
    b'{"version":1,"partitions":[{"topic":"b","weight":123456789012345678901234,"replicas":[4,5]}]}',
]


@pytest.mark.parametrize("i", range(len(EDGE)))
def test_edge_documents(i):
    same_as_dom(EDGE[i])


def test_fast_path_takes_the_common_shapes():
    # the documents the CLI normally sees never fall back to the DOM path
    for i in (0, 1, 4, 5, 6, 8, 26, 27, 28):
        assert cli.codec_roundtrip(EDGE[i], cli.CODEC_FAST)[0] == 0, EDGE[i]


def test_fuzzed_documents():
    base = json.dumps(synthetic(40, seed=9)).encode()
    rng = random.Random(1234)
    alphabet = b'{}[]:,"-.0123456789eEnul \\tx'
    for _ in range(400):
        b = bytearray(base)
        for _ in range(rng.randint(1, 3)):
            k = rng.randrange(len(b))
            op = rng.randrange(3)
            if op == 0:
                del b[k]
            elif op == 1:
                b.insert(k, rng.choice(alphabet))
            else:
                b[k] = rng.choice(alphabet)
        same_as_dom(bytes(b))


def test_float_formatting_matches_oracle():
    rng = random.Random(7)
    vals = [1e-6, 9.999999999999999e-7, 1e21, 9.99999999999999e20, 5e-324, 1.7976931348623157e308, 0.1, 123.456,
            -2.5e-9, 1e-7, 3.0, 100.0, 2 ** 53, 1.0 / 3.0]
    vals += [rng.uniform(-1, 1) * 10 ** rng.randint(-12, 25) for _ in range(300)]
    pl = {"version": 1, "partitions": [{"topic": "t", "partition": i, "replicas": [1], "weight": v}
                                       for i, v in enumerate(vals) if v != 0]}
    data = json.dumps(pl).encode()
    rc, got, *_ = cli.codec_roundtrip(data)
    code, want, err = O.run_plan(O.OraclePL(pl), O.default_cfg(), max_reassign=0, full_output=True)
    assert rc == 0 and code == 0, err
    assert got == want


@pytest.mark.parametrize("threads", ["2", "5", "16"])
@pytest.mark.parametrize("trap", ["none", "some", "all"])
def test_parallel_decode_matches_dom(threads, trap, monkeypatch):
    """The partitions array split over threads (codecs.cpp partitions_par): split points
    found inside topic strings that contain "},{" must not change the result -- the
    chunk-boundary proof rejects them and the one-thread pass decides."""
    monkeypatch.setenv("KB_CODEC_THREADS", threads)
    pl = synthetic(3000, seed=11)
    rng = random.Random(int(threads) * 7 + len(trap))
    for p in pl["partitions"]:
        if trap == "all" or (trap == "some" and rng.random() < 0.01):
            p["topic"] = p["topic"] + "},{topic:x" + "}, {" * rng.randint(0, 2)
    data = json.dumps(pl).encode()
    assert same_as_dom(data) == 0
    rc, got, *_ = cli.codec_roundtrip(data)
    code, want, err = O.run_plan(O.OraclePL(pl), O.default_cfg(), max_reassign=0, full_output=True)
    assert rc == 0 and code == 0 and got == want
    # whitespace between elements and a truncated document
    # (with traps the replacement also puts raw control bytes into topics: the DOM
    # parser rejects those, and the fast path must give up and agree)
    spaced = data.replace(b"}, {", b"} ,\n\t{")
    assert same_as_dom(spaced) == (0 if trap == "none" else 2)
    assert same_as_dom(data[: len(data) // 2]) != 0
