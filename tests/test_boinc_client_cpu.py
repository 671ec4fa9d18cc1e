"""The application binary under an in-repo fake BOINC client (tools/fake_boinc_client.py):
shared-memory heartbeat, process control (suspend / resume / quit / abort),
app status (fraction_done, CPU times), finish / temporary-exit markers, the
slot lock, and the crash / kill-signal paths (erp_boinc_wrapper.cpp:123-192,
495-573; erp_boinc_ipc.cpp:197-208; demod_binary.c:451-487, 1241-1296,
1420-1441, 1489-1492).

No BOINC client exists in this environment, so parity of the channel layout
and message texts with a real client is unpinned; what is pinned is the
behaviour the reference relies on: suspend pauses the work, quit leaves
without a final checkpoint, the result after quit + restart equals an
uninterrupted run."""
import fcntl
import os
import signal
import struct
import subprocess
import sys
import time
from pathlib import Path

import pytest

from boinc_app_eah_brp_amd.models.search import app_binary
from boinc_app_eah_brp_amd.utils import synth

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
from fake_boinc_client import FakeClient  # noqa: E402

N_TEMPLATES = 29  # bank lines (+1 injected template)
SLOW_MS = 120     # per-template pacing of the applier (BRP_FAULT=slow_template)


@pytest.fixture(scope="module")
def app(brp):
    p = app_binary()
    if not p.exists():
        from boinc_app_eah_brp_amd import _build

        _build.build()
    return p


@pytest.fixture(scope="module")
def case(tmp_path_factory):
    d = tmp_path_factory.mktemp("client_case")
    return synth.synthetic_case(d, n=1 << 13, n_templates=N_TEMPLATES,
                                inj=synth.Injection(f0=150.0, P_orb=900.0, tau=0.01, psi0=1.0, amplitude=3.0))


def _args(app, c, extra=()):
    return [app, "-i", c["wu"], "-t", c["bank"], "-l", c["zap"], "-o", "result.cand", "-c", "checkpoint.cpt",
            "-A", "0.08", "-P", "1.0", "-f", "400.0", "-W", "-B", "50", "--mi355x-cpu", *extra]


def _cands(path):
    return [l for l in Path(path).read_text().splitlines() if l and not l.startswith("%")]


@pytest.fixture(scope="module")
def reference_result(app, case, tmp_path_factory):
    d = tmp_path_factory.mktemp("uninterrupted")
    r = subprocess.run([str(a) for a in _args(app, case)], cwd=d, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _cands(d / "result.cand")
    assert lines
    return lines


def _slow_env(**kw):
    env = {"BRP_FAULT": f"slow_template:{SLOW_MS}", "BRP_CRASH_SLEEP": "0"}
    env.update(kw)
    return env


def test_status_suspend_resume_and_finish(app, case, reference_result, tmp_path):
    cl = FakeClient(tmp_path / "slot")
    try:
        cl.start(_args(app, case), env=_slow_env())
        cl.wait_fraction(0.2)
        cl.control("<suspend/>")
        time.sleep(0.6)  # the batch in flight finishes inside its critical section
        t_susp = time.time()
        f1 = cl.wait_status_after(t_susp)["fraction_done"]
        time.sleep(2.5)
        st = cl.wait_status_after(time.time())
        # status keeps flowing while suspended, progress does not
        assert st["fraction_done"] == f1, (f1, st)
        assert f1 < 0.9
        cl.control("<resume/>")
        rc, out, err = cl.wait()
    finally:
        cl.close()
    assert rc == 0, err[-3000:]
    slot = tmp_path / "slot"
    assert (slot / "boinc_finish_called").read_text().strip() == "0"
    assert (slot / "boinc_lockfile").exists()
    fr = [s["fraction_done"] for s in cl.statuses]
    assert fr == sorted(fr), fr
    assert fr[-1] == pytest.approx(1.0)
    assert all("current_cpu_time" in s and "checkpoint_cpu_time" in s for s in cl.statuses)
    assert max(s["checkpoint_cpu_time"] for s in cl.statuses) > 0
    assert "Received suspend message" in err and "Received resume message" in err
    assert _cands(slot / "result.cand") == reference_result
    text = (slot / "result.cand").read_text()
    assert "% User: 31 (volunteer)" in text and "% Host: 9 (0123456789abcdef)" in text


def test_quit_leaves_without_final_checkpoint_and_restart_matches(app, case, reference_result, tmp_path):
    slot = tmp_path / "slot"
    cl = FakeClient(slot)
    try:
        cl.start(_args(app, case), env=_slow_env())
        cl.wait_fraction(0.3)
        cl.control("<quit/>")
        rc, out, err = cl.wait(timeout=60)
    finally:
        cl.close()
    assert rc == 0, err[-3000:]
    assert "Received quit message" in err
    assert not (slot / "boinc_finish_called").exists()
    assert not (slot / "result.cand").exists()
    n_done = struct.unpack("<I", (slot / "checkpoint.cpt").read_bytes()[:4])[0]
    assert 0 < n_done < N_TEMPLATES + 1
    # the client restarts the task in the same slot: it resumes and finishes
    cl2 = FakeClient(slot)
    try:
        cl2.start(_args(app, case), env=_slow_env(BRP_FAULT="slow_template:5"))
        rc, out, err = cl2.wait()
    finally:
        cl2.close()
    assert rc == 0, err[-3000:]
    assert f"Continuing work on" in err
    assert (slot / "boinc_finish_called").read_text().strip() == "0"
    assert _cands(slot / "result.cand") == reference_result


def test_no_heartbeat_exits(app, case, tmp_path):
    cl = FakeClient(tmp_path / "slot")
    cl.heartbeat = False
    try:
        t0 = time.time()
        cl.start(_args(app, case), env=_slow_env(BRP_HEARTBEAT_GIVEUP="1.5"))
        rc, out, err = cl.wait(timeout=60)
    finally:
        cl.close()
    assert rc == 0
    assert time.time() - t0 < 0.5 + N_TEMPLATES * SLOW_MS / 1000.0
    assert "No heartbeat from the client" in err
    assert not (tmp_path / "slot" / "boinc_finish_called").exists()
    assert not (tmp_path / "slot" / "result.cand").exists()


def test_abort_exit_code(app, case, tmp_path):
    cl = FakeClient(tmp_path / "slot")
    try:
        cl.start(_args(app, case), env=_slow_env())
        cl.wait_fraction(0.1)
        cl.control("<abort/>")
        rc, out, err = cl.wait(timeout=60)
    finally:
        cl.close()
    assert rc == 194, err[-2000:]
    assert not (tmp_path / "slot" / "result.cand").exists()


def test_second_instance_in_slot_is_refused(app, case, tmp_path):
    slot = tmp_path / "slot"
    cl = FakeClient(slot)
    with open(slot / "boinc_lockfile", "w") as lk:
        fcntl.lockf(lk, fcntl.LOCK_EX | fcntl.LOCK_NB)
        try:
            cl.start(_args(app, case), env=_slow_env(BRP_LOCK_WAIT="0.5"))
            rc, out, err = cl.wait(timeout=60)
        finally:
            cl.close()
    assert rc == 0
    assert "Can't acquire lockfile" in err
    assert not (slot / "result.cand").exists()


def test_temporary_exit_marker(app, case, tmp_path):
    r = subprocess.run([str(a) for a in _args(app, case)], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, BRP_FAULT="resource_error"))
    assert r.returncode == 0, r.stderr[-2000:]
    marker = (tmp_path / "boinc_temporary_exit").read_text().splitlines()
    assert marker[0] == "900" and "Not enough free CPU/GPU memory" in marker[1]
    assert not (tmp_path / "boinc_finish_called").exists()


def test_segfault_prints_symbolised_backtrace_and_finishes(app, case, tmp_path):
    r = subprocess.run([str(a) for a in _args(app, case)], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, BRP_FAULT="segv_after_template:3", BRP_CRASH_SLEEP="0"))
    # finish(sig): exit status is the signal number, with the finish marker
    assert r.returncode == signal.SIGSEGV, r.stderr[-3000:]
    err = r.stderr
    assert "Application caught signal 11." in err
    assert "Backtrace:" in err and "End of backtrace" in err
    frames = [l for l in err.splitlines() if l.startswith("#")]
    assert any("brp::run_search" in l for l in frames), "\n".join(frames)
    assert any(" in main+" in l for l in frames), "\n".join(frames)
    assert (tmp_path / "boinc_finish_called").read_text().strip() == str(int(signal.SIGSEGV))


def test_kill_signals_ignored_three_times(app, case, tmp_path):
    p = subprocess.Popen([str(a) for a in _args(app, case)], cwd=tmp_path, stdout=subprocess.DEVNULL,
                         stderr=subprocess.PIPE, text=True, env=dict(os.environ, **_slow_env()))
    try:
        time.sleep(1.0)
        for _ in range(3):
            p.send_signal(signal.SIGTERM)
            time.sleep(0.2)
        assert p.poll() is None
        p.send_signal(signal.SIGINT)
        _, err = p.communicate(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == 0
    assert err.count("Application caught signal") == 4
    assert "Got 4th kill-signal" in err
    assert (tmp_path / "boinc_finish_called").read_text().strip() == "0"
    assert not (tmp_path / "result.cand").exists()


def test_tsan_under_client_suspend_resume_quit(case, reference_result, tmp_path):
    """Race detection with the client in the loop: the ThreadSanitizer build
    (_build.py --tsan) with two CPU workers, the runtime's status / control
    thread and the fake client's suspend, resume, then quit and restart. No
    ThreadSanitizer report, and the restarted task finishes with the
    uninterrupted result."""
    from boinc_app_eah_brp_amd import _build

    tsan = _build.build_tsan(verbose=False)
    env = _slow_env(TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    slot = tmp_path / "slot"
    cl = FakeClient(slot)
    try:
        cl.start(_args(tsan, case, ("--mi355x-gpus", "2")), env=env)
        cl.wait_fraction(0.2)
        cl.control("<suspend/>")
        time.sleep(0.6)
        cl.control("<resume/>")
        cl.wait_fraction(0.4)
        cl.control("<quit/>")
        rc, out, err = cl.wait(timeout=120)
    finally:
        cl.close()
    assert rc == 0 and "ThreadSanitizer" not in err, err[-6000:]
    cl2 = FakeClient(slot)
    try:
        cl2.start(_args(tsan, case, ("--mi355x-gpus", "2")), env=dict(env, BRP_FAULT="slow_template:5"))
        rc, out, err = cl2.wait(timeout=180)
    finally:
        cl2.close()
    assert rc == 0 and "ThreadSanitizer" not in err, err[-6000:]
    assert _cands(slot / "result.cand") == reference_result


def _children(pid):
    try:
        return [int(x) for x in Path(f"/proc/{pid}/task/{pid}/children").read_text().split()]
    except OSError:
        return []


def _alive(pid):
    try:
        st = Path(f"/proc/{pid}/stat").read_text().split(") ")[-1].split()[0]
    except OSError:
        return False
    return st != "Z"


def test_supervised_run_equals_unsupervised(app, case, reference_result, tmp_path):
    """BRP_SUPERVISE (default on): the parent the client waits for leaves with
    the child's status; results, markers and exit codes are those of an
    unsupervised run (BRP_SUPERVISE=0)."""
    for sup in ("1", "0"):
        d = tmp_path / f"sup{sup}"
        d.mkdir()
        r = subprocess.run([str(a) for a in _args(app, case)], cwd=d, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, BRP_SUPERVISE=sup))
        assert r.returncode == 0, r.stderr[-2000:]
        assert _cands(d / "result.cand") == reference_result
        assert (d / "boinc_finish_called").read_text().strip() == "0"
    # a fatal signal in the worker: same exit status either way
    codes = []
    for sup in ("1", "0"):
        d = tmp_path / f"segv{sup}"
        d.mkdir()
        r = subprocess.run([str(a) for a in _args(app, case)], cwd=d, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, BRP_SUPERVISE=sup, BRP_FAULT="segv_after_template:3",
                                    BRP_CRASH_SLEEP="0"))
        codes.append(r.returncode)
    assert codes[0] == codes[1] == signal.SIGSEGV


def test_supervisor_parent_death_kills_child(app, case, tmp_path):
    """SIGKILL of the parent (the client's hard kill) takes the worker child
    with it (PR_SET_PDEATHSIG): no orphan keeps the GPU."""
    p = subprocess.Popen([str(a) for a in _args(app, case)], cwd=tmp_path, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, env=dict(os.environ, **_slow_env()))
    try:
        kids = []
        for _ in range(100):
            kids = _children(p.pid)
            if kids:
                break
            time.sleep(0.05)
        assert len(kids) == 1, "the supervised app runs its work in one child"
        child = kids[0]
        time.sleep(0.5)
        assert _alive(child)
        p.kill()
        p.wait(timeout=10)
        for _ in range(100):
            if not _alive(child):
                break
            time.sleep(0.05)
        assert not _alive(child), "worker child survived its parent"
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()


def test_supervisor_parent_leaves_before_child_teardown(app, case, tmp_path):
    """The parent exits once the child has reported (results and the finish
    marker on disk), not when the child is gone: BRP_FAULT=slow_exit holds the
    child 3 s after its report, as the GPU context's teardown does for ~0.1 s
    (the parent's exit then ends the delay: PR_SET_PDEATHSIG)."""
    t0 = time.perf_counter()
    p = subprocess.Popen([str(a) for a in _args(app, case)], cwd=tmp_path, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, env=dict(os.environ, BRP_FAULT="slow_exit:3000"))
    rc = p.wait(timeout=120)
    t_parent = time.perf_counter() - t0
    assert rc == 0
    assert (tmp_path / "boinc_finish_called").read_text().strip() == "0"
    assert _cands(tmp_path / "result.cand")
    # unsupervised, the same run waits for the delay
    d = tmp_path / "unsup"
    d.mkdir()
    t1 = time.perf_counter()
    r = subprocess.run([str(a) for a in _args(app, case)], cwd=d, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       env=dict(os.environ, BRP_FAULT="slow_exit:3000", BRP_SUPERVISE="0"), timeout=120)
    assert r.returncode == 0
    assert time.perf_counter() - t1 >= 3.0 > t_parent + 1.0
