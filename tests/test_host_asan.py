"""Memory and thread safety of the C++ host runtime on CPU: the session /
sim driver (tests/cpp/nulldev/session_asan.cpp) and the party-process
drivers compiled with the host sources under AddressSanitizer and
ThreadSanitizer, linked against a host-memory stand-in for libaby3gpu.so
(gen_nulldev.py) that performs no compute. Covers the scheduler, channels
(copying and zero-copy), the cross-process links, the stream-ordered pools
and their cross-party fences, and session teardown. With ND_ASYNC=1 the
stand-in's streams run asynchronously (a thread each, random delays), so the
host's stream-ordering rules are exercised as on a device."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ND = os.path.join(ROOT, "tests", "cpp", "nulldev")


_OBJS = {}  # sanitizer -> object files of the host sources + the null device (built once per session)


def _objects(sanitizer):
    """The host runtime's sources and the null device compiled once per
    sanitizer (in parallel), shared by every driver of this module."""
    if sanitizer in _OBJS:
        return _OBJS[sanitizer]
    import tempfile
    from concurrent.futures import ThreadPoolExecutor

    out = tempfile.mkdtemp(prefix=f"nd_{sanitizer}_")
    nulldev = os.path.join(out, "nulldev.cpp")
    subprocess.run([sys.executable, os.path.join(ND, "gen_nulldev.py"), nulldev], check=True)
    srcs = sorted(glob.glob(os.path.join(ROOT, "aby3_amd", "host", "*.cpp"))) + [nulldev]

    def cc(src):
        obj = os.path.join(out, os.path.basename(src)[:-4] + ".o")
        subprocess.run(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer",
                        "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "aby3_amd", "host"),
                        "-c", src, "-o", obj], check=True, timeout=600)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        _OBJS[sanitizer] = list(ex.map(cc, srcs))
    return _OBJS[sanitizer]


def _build(tmp, sanitizer, driver="session_asan.cpp"):
    exe = os.path.join(tmp, f"{driver[:-4]}_{sanitizer}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer",
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "aby3_amd", "host"),
           *_objects(sanitizer), os.path.join(ND, driver), "-o", exe, "-pthread", "-lrt"]
    subprocess.run(cmd, check=True, timeout=600)
    return exe


@pytest.mark.parametrize("sanitizer,nd_async", [("address", "0"), ("thread", "0"), ("address", "1")])
def test_host_runtime_sanitized(tmp_path, sanitizer, nd_async):
    exe = _build(str(tmp_path), sanitizer)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", TSAN_OPTIONS="halt_on_error=1", ND_ASYNC=nd_async)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "session_asan: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


@pytest.mark.parametrize("sanitizer,nd_async", [("address", "0"), ("thread", "0"), ("address", "1")])
def test_party_processes_sanitized(tmp_path, sanitizer, nd_async):
    """Three processes, one party each (aby3h_party_create): every job over
    the shared-memory links and IPC staging slots in the three layouts, under
    AddressSanitizer and ThreadSanitizer (each process's party thread, link
    writer threads and link watchdog)."""
    exe = _build(str(tmp_path), sanitizer, "party_procs.cpp")
    # 1 MiB hand-off arenas: the null device's shared memory is a bump allocator
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", TSAN_OPTIONS="halt_on_error=1",
               ABY3_LINK_TIMEOUT_S="60", ABY3_ARENA_MB="1", ND_ASYNC=nd_async)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "party_procs: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


def test_party_failure_ends_peers_fast(tmp_path):
    """One party per process, party 1 failing (a failed copy during its setup;
    its process gone right after the ring is built): both peers exit non-zero
    within 2 s, naming party 1's error or its exit (a
    setup failure used to cost the peers the full link timeout)."""
    exe = _build(str(tmp_path), "address", "party_fail.cpp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", ABY3_LINK_TIMEOUT_S="60")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "party_fail: ok" in r.stdout, r.stdout
    out = r.stdout
    # mode 1: the peers name party 1's own error through the abort word
    assert out.count("failed: party 1 setup") >= 2, out
    # mode 2: the watchdog finds party 1's process gone without closing
    assert out.count("exited without closing link") >= 2, out


def test_pool_trim(tmp_path):
    """The stream-ordered pool: trim() empties a cache of mixed size classes
    and allocation goes on; a session past ABY3_POOL_TRIM_MB trims its
    parties' pools between runs."""
    exe = _build(str(tmp_path), "address", "pool_trim.cpp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "pool_trim: ok" in r.stdout, r.stdout


def test_link_staging_slots_async(tmp_path):
    """The staging slots' ordering and lifetime rules (Channel.cpp) on the
    null device with asynchronous streams (ND_ASYNC=1): 1200 device messages
    per direction across the slots' size steps, by all three send forms,
    completed out of order while later sends reuse and outgrow slots; every
    message's bytes are checked and a copy through a closed IPC mapping
    aborts. Dropping the sender's wait for the receiver's copy-out, or closing
    a replaced mapping without waiting for the copy-outs behind it, makes
    this test fail (checked by hand against both mutations)."""
    exe = _build(str(tmp_path), "address", "link_slots.cpp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", ABY3_LINK_TIMEOUT_S="60", ND_ASYNC="1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "link_slots: ok" in r.stdout, r.stdout


def test_link_large_cyclic_exchange(tmp_path):
    """Three processes, each sending host payloads of three times a link's
    ring size to the next party before receiving from the previous one
    (this cycle used to block until the link timeout)."""
    exe = _build(str(tmp_path), "address", "link_exchange.cpp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", ABY3_LINK_TIMEOUT_S="30")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "link_exchange: ok" in r.stdout


@pytest.mark.parametrize("sanitizer", ["address", "thread"])
def test_device_batch_sampler(tmp_path, sanitizer):
    """DeviceBatchSampler (getSubset with the pool in device memory and the
    reshuffle on a host thread) yields BatchSampler's mini-batches exactly."""
    exe = _build(str(tmp_path), sanitizer, "sampler_check.cpp")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "sampler_check: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
