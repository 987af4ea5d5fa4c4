"""The reference's CLI tests (kafkabalancer_test.go:11-166) on the native CLI,
plus byte-exact plan output against the oracle's run() restatement."""
import os

import pytest

from kafkabalancer_amd import cli
from oracle import oracle as O

from helpers import GOLDEN, golden

TEST_JSON = os.path.join(GOLDEN, "test.json")
with open(TEST_JSON, "rb") as f:
    TEST_BYTES = f.read()


def test_main_help():                                    # kafkabalancer_test.go:11
    rc, _, err = cli.run(["kafkabalancer", "-help"], TEST_BYTES)
    assert rc == 0 and "Usage of kafkabalancer:" in err


def test_main_file_and_zk():                             # :40
    rc, _, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON, "-from-zk=localhost:2282"])
    assert rc == 3 and "can't specify both -input and -from-zk" in err


def test_main_partition_list_empty():                    # :51
    rc, _, err = cli.run(["kafkabalancer", "-input-json"], b"")
    assert rc == 2 and "failed getting partition list:" in err


def test_main_partition_list_malformed():                # :62
    rc, _, err = cli.run(["kafkabalancer", "-input-json"], b"::malformed::")
    assert rc == 2 and "failed getting partition list:" in err


def test_main_file_missing():                            # :73
    rc, _, _ = cli.run(["kafkabalancer", "-input-json", "-input=test/missing.json"])
    assert rc == 1


def test_main_broker_list_malformed():                   # :89
    rc, _, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON, "-broker-ids=malformed"])
    assert rc == 3 and "failed parsing broker list" in err


def test_main_max_reassign_malformed():                  # :100
    rc, _, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON, "-max-reassign=-1"])
    assert rc == 3 and "invalid number of max reassignments" in err


def test_broken_zk_conn_string():                        # :145
    rc, _, err = cli.run(["kafkabalancer", "-from-zk=."])
    assert rc == 2 and "failed parsing zk connection string" in err


def test_text_and_json_parse_errors():
    rc, _, err = cli.run(["kafkabalancer", "-input-json"], b'{"version":2,"partitions":[]}')
    assert rc == 2 and "wrong partition list version: expected 1, got 2" in err
    rc, _, err = cli.run(["kafkabalancer", "-input-json"], b'{"version":1,"partitions":[{"topic":"a","partition":1.5}]}')
    assert rc == 2 and "cannot unmarshal number 1.5" in err
    rc, _, err = cli.run(["kafkabalancer"], b"no matching lines\n")
    assert rc == 2 and "empty partition list" in err


# ------------------------------------------------------------- GPU cases

@pytest.mark.gpu
def test_main_stdin_and_file():                          # :23, :32
    rc, out, _ = cli.run(["kafkabalancer", "-input-json"], TEST_BYTES)
    assert rc == 0
    rc2, out2, _ = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON])
    assert rc2 == 0 and out == out2


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["-broker-ids=1,2,3"], ["-max-reassign=1000"], ["-full-output"]])
def test_main_flags_ok(args):                            # :78, :111, :119
    rc, _, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON] + args)
    assert rc == 0, err


@pytest.mark.gpu
def test_broken_output_stream():                         # :127-143
    rc, _, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON], fail_output=True)
    assert rc == 4 and "failed writing partition list" in err


@pytest.mark.gpu
def test_broken_data():                                  # :156
    j = b'{"version":1,"partitions":[{"topic":"foo1","partition":1,"replicas":[1,2],"num_replicas":3}]}'
    rc, _, err = cli.run(["kafkabalancer", "-input-json"], j)
    assert rc == 3 and "unable to pick replica to add" in err


CLI_VARIANTS = [
    ([], {}),
    (["-max-reassign=1000"], dict(max_reassign=1000)),
    (["-full-output"], dict(full_output=True)),
    (["-max-reassign=5", "-complete-partition=false"], dict(max_reassign=5, complete_partition=False)),
    (["-allow-leader", "-max-reassign=8", "-complete-partition=false"],
     dict(max_reassign=8, complete_partition=False, cfg=dict(allow_leader=True))),
    (["-allow-leader", "-max-reassign=8", "-complete-partition=false", "-unique"],
     dict(max_reassign=8, complete_partition=False, unique=True, cfg=dict(allow_leader=True))),
    (["-broker-ids=1,2,3,4,5,6", "-max-reassign=20"], dict(max_reassign=20, cfg=dict(brokers=[1, 2, 3, 4, 5, 6]))),
    (["-rebalance-leader", "-min-unbalance=0", "-max-reassign=6", "-complete-partition=false"],
     dict(max_reassign=6, complete_partition=False, cfg=dict(rebalance_leaders=True, min_unbalance=0.0))),
    # a budget far beyond any plan: the planner runs in bounded chunks until no change
    # (non-leader moves: -allow-leader plans can cycle forever, as in the reference)
    (["-min-unbalance=0", "-max-reassign=1000000000", "-complete-partition=false"],
     dict(max_reassign=1000000000, complete_partition=False, cfg=dict(min_unbalance=0.0))),
]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", range(len(CLI_VARIANTS)))
def test_cli_output_bytes_match_oracle(variant):
    args, kw = CLI_VARIANTS[variant]
    kw = dict(kw)
    cfg = O.default_cfg()
    cfg.update(kw.pop("cfg", {}))
    code, want, _ = O.run_plan(O.OraclePL(golden("test.json")), cfg, sem=O.SEM_GO, **kw)
    rc, out, err = cli.run(["kafkabalancer", "-input-json", "-input=" + TEST_JSON] + args)
    assert rc == code, err
    assert out == want, (out, want)


@pytest.mark.gpu
def test_cli_text_input():
    text = ("Topic:test\tPartitionCount:3\tReplicationFactor:3\tConfigs:\n"
            "\tTopic: test\tPartition: 0\tLeader: 2\tReplicas: 2,0,1\tIsr: 0,1,2\n"
            "\tTopic: test\tPartition: 1\tLeader: 0\tReplicas: 0,1,2\tIsr: 0,1,2\n"
            "\tTopic: other\tPartition: 2\tLeader: 1\tReplicas: 1,2,0,3\tIsr: 0,1,2\n")
    rc, out, err = cli.run(["kafkabalancer", "-topics=test,other", "-max-reassign=3"], text.encode())
    assert rc == 0, err
    plist = {"version": 1, "partitions": [
        {"topic": "test", "partition": 0, "replicas": [2, 0, 1]},
        {"topic": "test", "partition": 1, "replicas": [0, 1, 2]},
        {"topic": "other", "partition": 2, "replicas": [1, 2, 0, 3]}]}
    code, want, _ = O.run_plan(O.OraclePL(plist), O.default_cfg(), max_reassign=3)
    assert out == want
