"""The known-answer tests of tests/test_kat.py, run on the HIP engine."""
import pytest

import kat_scenarios as K

pytestmark = pytest.mark.gpu

VOTER = K.load("kat_voter.json")
MSGAPP = K.load("kat_check_msgapp.json")
APPEND = K.load("kat_append.json")
FIG7 = K.load("kat_figure7.json")
CTC = K.load("kat_current_term_commit.json")
QC = K.load("kat_quorum_commit.json")


@pytest.mark.parametrize("case", VOTER["cases"])
def test_voter_up_to_date(case):
    assert K.run_voter("gpu", case) == case["reject"]


@pytest.mark.parametrize("case", MSGAPP["cases"])
def test_follower_check_msgapp(case):
    got = K.run_check_msgapp("gpu", MSGAPP, case)
    assert got == dict(reject=case["reject"], resp_index=case["resp_index"], hint=case["hint"])


@pytest.mark.parametrize("case", APPEND["cases"])
def test_follower_append_entries(case):
    assert K.run_append("gpu", APPEND, case) == case["want"]


def test_figure7_convergence():
    logs, views = K.run_figure7("gpu", FIG7)
    for lg in logs:
        assert lg == FIG7["want_log"]
    assert all(v["committed"] == FIG7["want_commit"] for v in views)


def test_leader_only_commits_current_term():
    assert K.run_current_term_commit("gpu", CTC) == [a["want_commit"] for a in CTC["acks"]]


@pytest.mark.parametrize("case", QC["cases"])
def test_quorum_commit(case):
    assert K.run_quorum_commit("gpu", case) == case["committed"]


@pytest.mark.parametrize("name", sorted(K.PAPER_KATS))
def test_paper_kats(name):
    """The etcd paper-test shapes through rg_import_replica / rg_deliver / rg_tick."""
    assert all(K.PAPER_KATS[name]("gpu"))


def test_term_limit():
    """The 36-bit term boundary: the engine refuses a campaign at 2^36 - 1 exactly as the oracles do."""
    assert K.run_term_limit("gpu", K.TERM_MAX - 1) == ("candidate", K.TERM_MAX, 0, 2)
    assert K.run_term_limit("gpu", K.TERM_MAX) == ("follower", K.TERM_MAX, K.ERR_TERM_LIMIT, 0)
    assert K.run_term_limit("c", K.TERM_MAX) == K.run_term_limit("gpu", K.TERM_MAX)
