"""Known-answer tests on both CPU restatements (C oracle and pyraft)."""
import pytest

import kat_scenarios as K
from engines import KINDS_CPU

VOTER = K.load("kat_voter.json")
MSGAPP = K.load("kat_check_msgapp.json")
APPEND = K.load("kat_append.json")
FIG7 = K.load("kat_figure7.json")
CTC = K.load("kat_current_term_commit.json")
QC = K.load("kat_quorum_commit.json")


@pytest.mark.parametrize("kind", KINDS_CPU)
@pytest.mark.parametrize("case", VOTER["cases"], ids=lambda c: f"{c['log']}-{c['cand_log_term']},{c['cand_index']}")
def test_voter_up_to_date(kind, case):
    assert K.run_voter(kind, case) == case["reject"]


@pytest.mark.parametrize("kind", KINDS_CPU)
@pytest.mark.parametrize("case", MSGAPP["cases"], ids=lambda c: f"{c['log_term']},{c['log_index']}")
def test_follower_check_msgapp(kind, case):
    got = K.run_check_msgapp(kind, MSGAPP, case)
    assert got == dict(reject=case["reject"], resp_index=case["resp_index"], hint=case["hint"])


@pytest.mark.parametrize("kind", KINDS_CPU)
@pytest.mark.parametrize("case", APPEND["cases"], ids=lambda c: f"{c['log_index']}-{c['entries']}")
def test_follower_append_entries(kind, case):
    assert K.run_append(kind, APPEND, case) == case["want"]


@pytest.mark.parametrize("kind", KINDS_CPU)
def test_figure7_convergence(kind):
    logs, views = K.run_figure7(kind, FIG7)
    for lg in logs:
        assert lg == FIG7["want_log"]
    assert views[0]["role"] == 2 and views[0]["term"] == FIG7["leader_term"]
    assert all(v["committed"] == FIG7["want_commit"] for v in views)
    assert all(v["err"] == 0 for v in views)


@pytest.mark.parametrize("kind", KINDS_CPU)
def test_leader_only_commits_current_term(kind):
    assert K.run_current_term_commit(kind, CTC) == [a["want_commit"] for a in CTC["acks"]]


@pytest.mark.parametrize("kind", KINDS_CPU)
@pytest.mark.parametrize("case", QC["cases"], ids=lambda c: f"n{c['size']}-{c['acceptors']}")
def test_quorum_commit(kind, case):
    assert K.run_quorum_commit(kind, case) == case["committed"]


@pytest.mark.parametrize("kind", KINDS_CPU)
@pytest.mark.parametrize("name", sorted(K.PAPER_KATS))
def test_paper_kats(kind, name):
    """etcd raft paper-test shapes (leader election, candidate fallback, term update, leader and
    follower commit, vote request, CheckQuorum step-down); parity with dragonboat unpinned."""
    assert all(K.PAPER_KATS[name](kind))


@pytest.mark.parametrize("kind", KINDS_CPU)
def test_term_limit(kind):
    assert K.run_term_limit(kind, K.TERM_MAX - 1) == ("candidate", K.TERM_MAX, 0, 2)
    assert K.run_term_limit(kind, K.TERM_MAX) == ("follower", K.TERM_MAX, K.ERR_TERM_LIMIT, 0)
