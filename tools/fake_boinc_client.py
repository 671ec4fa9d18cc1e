"""A minimal in-repo BOINC client for driving the application binary in a slot
directory (no real client is available here, so parity with one is unpinned).

It does what the client side of the app protocol does (csrc/boinc/client_shm.hpp):
writes init_data.xml, creates the 8 KB `boinc_mmap_file`, sends `<heartbeat/>`
every 0.5 s, posts process-control messages (`<suspend/>`, `<resume/>`,
`<quit/>`, `<abort/>`) and reads the app status the app posts once a second.

    client = FakeClient(slot_dir)
    client.start([app, "-i", ...])
    client.wait_fraction(0.3)
    client.control("<suspend/>")
"""
from __future__ import annotations

import mmap
import os
import re
import subprocess
import threading
import time
from pathlib import Path

CHANNEL = 1024
CHANNELS = ("process_control_request", "process_control_reply", "graphics_request", "graphics_reply", "heartbeat",
            "app_status", "trickle_up", "trickle_down")
SHM_SIZE = CHANNEL * len(CHANNELS)


class FakeClient:
    def __init__(self, slot: str | Path, checkpoint_period: float = 0.0, extra_init: str = ""):
        self.slot = Path(slot)
        self.slot.mkdir(parents=True, exist_ok=True)
        (self.slot / "init_data.xml").write_text(
            "<app_init_data>\n<major_version>7</major_version>\n<userid>31</userid>\n<user_name>volunteer</user_name>\n"
            "<hostid>9</hostid>\n<host_cpid>0123456789abcdef</host_cpid>\n<slot>0</slot>\n"
            f"<wu_name>brp_test_wu</wu_name>\n<checkpoint_period>{checkpoint_period}</checkpoint_period>\n"
            f"{extra_init}</app_init_data>\n")
        path = self.slot / "boinc_mmap_file"
        path.write_bytes(b"\0" * SHM_SIZE)
        self._f = open(path, "r+b")
        self.shm = mmap.mmap(self._f.fileno(), SHM_SIZE)
        self.proc: subprocess.Popen | None = None
        self.statuses: list[dict] = []
        self.heartbeat = True
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._lock = threading.Lock()

    # ---- channels -------------------------------------------------------------
    def _off(self, name: str) -> int:
        return CHANNELS.index(name) * CHANNEL

    def send(self, name: str, msg: str) -> bool:
        o = self._off(name)
        with self._lock:
            if self.shm[o] != 0:
                return False
            data = msg.encode()[: CHANNEL - 2] + b"\0"
            self.shm[o + 1:o + 1 + len(data)] = data
            self.shm[o] = 1
        return True

    def receive(self, name: str) -> str | None:
        o = self._off(name)
        with self._lock:
            if self.shm[o] == 0:
                return None
            raw = bytes(self.shm[o + 1:o + CHANNEL])
            self.shm[o] = 0
        return raw.split(b"\0", 1)[0].decode()

    def control(self, msg: str, timeout: float = 10.0) -> None:
        t0 = time.time()
        while not self.send("process_control_request", msg):
            if time.time() - t0 > timeout:
                raise TimeoutError(f"process_control_request still full, cannot send {msg}")
            time.sleep(0.02)

    # ---- app lifetime -----------------------------------------------------------
    def start(self, argv: list[str], env: dict | None = None) -> subprocess.Popen:
        self._out = open(self.slot / "stdout.txt", "w")
        self._err = open(self.slot / "stderr.txt", "w")
        self.proc = subprocess.Popen([str(a) for a in argv], cwd=self.slot, env=dict(os.environ, **(env or {})),
                                     stdout=self._out, stderr=self._err, text=True)
        self._stop.clear()
        self._thread = threading.Thread(target=self._service, daemon=True)
        self._thread.start()
        return self.proc

    def _service(self) -> None:
        last_hb = 0.0
        while not self._stop.is_set():
            now = time.time()
            if self.heartbeat and now - last_hb >= 0.5:
                self.send("heartbeat", "<heartbeat/>\n<wss>1.5e8</wss>\n<max_wss>2.0e8</max_wss>\n")
                last_hb = now
            msg = self.receive("app_status")
            if msg is not None:
                st = {k: float(v) for k, v in re.findall(r"<(\w+)>([^<]+)</\1>", msg)}
                st["t"] = now
                self.statuses.append(st)
            if self.proc is not None and self.proc.poll() is not None:
                # drain a final status the app posted just before exiting
                msg = self.receive("app_status")
                if msg is not None:
                    st = {k: float(v) for k, v in re.findall(r"<(\w+)>([^<]+)</\1>", msg)}
                    st["t"] = time.time()
                    self.statuses.append(st)
                break
            time.sleep(0.05)

    def fraction(self) -> float:
        return self.statuses[-1]["fraction_done"] if self.statuses else 0.0

    def wait_fraction(self, f: float, timeout: float = 60.0) -> float:
        t0 = time.time()
        while self.fraction() < f:
            if self.proc.poll() is not None:
                raise RuntimeError(f"app exited ({self.proc.returncode}) before fraction {f}")
            if time.time() - t0 > timeout:
                raise TimeoutError(f"fraction_done stayed at {self.fraction()}")
            time.sleep(0.05)
        return self.fraction()

    def wait_status_after(self, t: float, timeout: float = 10.0) -> dict:
        t0 = time.time()
        while not self.statuses or self.statuses[-1]["t"] <= t:
            if time.time() - t0 > timeout:
                raise TimeoutError("no app status message")
            time.sleep(0.05)
        return self.statuses[-1]

    def wait(self, timeout: float = 120.0) -> tuple[int, str, str]:
        self.proc.wait(timeout=timeout)
        # the service thread drains the final status once it sees the exit
        if self._thread is not None:
            self._thread.join(timeout=5)
        self._stop.set()
        self._out.close()
        self._err.close()
        return (self.proc.returncode, (self.slot / "stdout.txt").read_text(),
                (self.slot / "stderr.txt").read_text())

    def close(self) -> None:
        self._stop.set()
        if self.proc is not None and self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()
        self.shm.close()
        self._f.close()
