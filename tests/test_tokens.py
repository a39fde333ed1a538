"""The pipelined-grid admission tokens (coll_comm.cpp: per-GPU tokens in a per-user shared-memory
table that outlives jobs) must not outlive their holders: a process killed while it holds a token
(SIGKILL, the OOM killer) would otherwise leave that GPU on the two-phase flow for every later job.
These run the holder protocol on the CPU through the test hook mi355x_debug_token (a private table
per test, MI355X_TOKEN_TABLE), with real processes killed mid-hold."""
from __future__ import annotations

import os
import pathlib
import signal
import subprocess
import sys
import time
import uuid

import pytest

REPO = pathlib.Path(__file__).resolve().parent.parent

# a process that takes (or tries) the token of device uid `uid` for communicator `name`, prints the
# outcome, then obeys stdin: "release", "exit", or nothing (it sleeps until killed)
CHILD = r"""
import ctypes, sys
sys.path.insert(0, {repo!r})
import __graft_entry__ as g
pkg = g._load_pkg()
lib = pkg.rt()
uid, name = int(sys.argv[1]), sys.argv[2].encode()
print("held" if lib.mi355x_debug_token(uid, name, 1) == 1 else "refused", flush=True)
for line in sys.stdin:
    cmd = line.strip()
    if cmd == "take":
        print("held" if lib.mi355x_debug_token(uid, name, 1) == 1 else "refused", flush=True)
    elif cmd == "release":
        lib.mi355x_debug_token(uid, name, 0)
        print("released", flush=True)
    elif cmd == "exit":
        break
"""


@pytest.fixture
def table(monkeypatch):
    name = "/mi355x_test_tokens_" + uuid.uuid4().hex[:12]
    monkeypatch.setenv("MI355X_TOKEN_TABLE", name)
    yield name
    try:
        os.unlink("/dev/shm" + name)
    except FileNotFoundError:
        pass


def _spawn(uid: int, name: str):
    p = subprocess.Popen([sys.executable, "-c", CHILD.format(repo=str(REPO)), str(uid), name], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    return p, p.stdout.readline().strip()


def _cmd(p, cmd: str) -> str:
    p.stdin.write(cmd + "\n")
    p.stdin.flush()
    return p.stdout.readline().strip()


def _finish(p):
    try:
        p.stdin.write("exit\n")
        p.stdin.flush()
    except BrokenPipeError:
        pass
    p.wait(30)
    return p.stderr.read()


def test_killed_holder_token_is_reclaimed(table):
    """a live holder refuses another communicator; once it is SIGKILLed (and reaped) the next one
    takes the token back, and says so"""
    uid = 0x5eed0001
    a, st = _spawn(uid, "commA")
    assert st == "held"
    b, st = _spawn(uid, "commB")
    assert st == "refused", "a live holder keeps its token"
    a.send_signal(signal.SIGKILL)
    a.wait(30)
    assert _cmd(b, "take") == "held", "the dead holder's token was not reclaimed"
    err = _finish(b)
    assert "reclaimed" in err


def test_zombie_holder_counts_as_dead(table):
    """a holder that exited without releasing but is not reaped yet (a zombie) is gone"""
    uid = 0x5eed0002
    a, st = _spawn(uid, "commA")
    assert st == "held"
    a.stdin.write("exit\n")
    a.stdin.flush()
    time.sleep(1.0)  # exited; not waited for: a zombie of this process
    b, st = _spawn(uid, "commB")
    assert st == "held", "an exited (zombie) holder should not keep its token"
    _finish(b)
    a.wait(30)


def test_shared_holder_survives_one_death(table):
    """ranks of ONE communicator sharing a GPU count up the same token: killing one of them must not
    free the token while the other still holds it; after the survivor releases, it is free"""
    uid = 0x5eed0003
    r0, st0 = _spawn(uid, "commA")
    r1, st1 = _spawn(uid, "commA")
    assert st0 == st1 == "held"
    r0.send_signal(signal.SIGKILL)
    r0.wait(30)
    other, st = _spawn(uid, "commB")
    assert st == "refused", "a live rank of the holding communicator still holds the token"
    assert _cmd(r1, "release") == "released"
    # the survivor gave its count back; the dead rank's count is taken back by the next taker
    assert _cmd(other, "take") == "held"
    _finish(other)
    _finish(r1)


def test_release_frees_for_others(table):
    """an ordinary release: the next communicator takes the token without any reclaim"""
    uid = 0x5eed0004
    a, st = _spawn(uid, "commA")
    assert st == "held"
    b, st = _spawn(uid, "commB")
    assert st == "refused"
    assert _cmd(a, "release") == "released"
    assert _cmd(b, "take") == "held"
    err = _finish(b)
    assert "reclaimed" not in err
    _finish(a)


def test_ranks_of_one_communicator_race_to_reclaim(table):
    """after the holder dies, several ranks of the next communicator try at once: one of them takes
    the token back, the others count up behind it -- none is refused (a rank that lost the race to
    reclaim must look at the token again, not give up)"""
    uid = 0x5eed0005
    for _ in range(5):
        a, st = _spawn(uid, "commA")
        assert st == "held"
        a.send_signal(signal.SIGKILL)
        a.wait(30)
        ranks = [subprocess.Popen([sys.executable, "-c", CHILD.format(repo=str(REPO)), str(uid), "commB"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
                 for _ in range(4)]
        states = [p.stdout.readline().strip() for p in ranks]
        assert states == ["held"] * 4, states
        for p in ranks:
            assert _cmd(p, "release") == "released"
            _finish(p)
