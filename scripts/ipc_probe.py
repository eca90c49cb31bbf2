"""IPC probe: process A allocates staging-sized buffers with aby3g_malloc in
two phases and exports their handles; process B opens phase 1's, closes two
of them, then opens phase 2's (allocated by A after B's closes, next to the
first ones), and copies from every live mapping. Reports failures: whether
an IPC mapping of a sub-allocated block survives its neighbours' opens and
closes (the staged-copy slots of Channel.cpp do exactly this)."""
import ctypes
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lib():
    from aby3_amd import native as nt
    return nt.lib()


def wait(path):
    while not os.path.exists(path):
        time.sleep(0.02)


def export(g, sizes, path):
    hs = []
    for sz in sizes:
        p = ctypes.c_void_p()
        g.malloc(ctypes.byref(p), sz)
        g.memset(p, 0x5A, sz, None)
        h = (ctypes.c_uint8 * 64)()
        g.ipc_get_handle(p, h)
        hs.append((sz, p.value, bytes(h)))
    g.device_sync()
    with open(path + ".tmp", "wb") as f:
        for sz, pv, h in hs:
            f.write(sz.to_bytes(8, "little") + pv.to_bytes(8, "little") + h)
    os.rename(path + ".tmp", path)
    return hs


def read(path):
    data = open(path, "rb").read()
    return [(int.from_bytes(data[i:i + 8], "little"), int.from_bytes(data[i + 8:i + 16], "little"),
             data[i + 16:i + 80]) for i in range(0, len(data), 80)]


def main():
    role, path = sys.argv[1], sys.argv[2]
    g = lib()
    if role == "A":
        a1 = export(g, [64 << 10] * 4 + [128 << 10] * 2, path + ".1")
        wait(path + ".closed")
        a2 = export(g, [64 << 10] * 2 + [128 << 10] * 2 + [256 << 10], path + ".2")
        wait(path + ".done")
        print("A phase 1", [hex(x[1]) for x in a1])
        print("A phase 2", [hex(x[1]) for x in a2])
        return
    fails = 0
    live = []

    def open_all(entries, tag):
        nonlocal fails
        for sz, pv, hb in entries:
            h = (ctypes.c_uint8 * 64).from_buffer_copy(hb)
            p = ctypes.c_void_p()
            try:
                g.ipc_open(h, ctypes.byref(p))
                live.append((sz, p.value))
                print(" ", tag, "open", hex(pv), "->", hex(p.value))
            except Exception as e:
                fails += 1
                print(" ", tag, "open", hex(pv), "FAIL", str(e)[:120])

    wait(path + ".1")
    open_all(read(path + ".1"), "p1")
    for k in (1, 4):  # close two openings (as the receiver does for replaced slots)
        sz, pv = live[k]
        g.ipc_close(ctypes.c_void_p(pv))
        print("  close", hex(pv))
    live = [x for i, x in enumerate(live) if i not in (1, 4)]
    open(path + ".closed", "w").write("x")
    wait(path + ".2")
    open_all(read(path + ".2"), "p2")
    dst = ctypes.c_void_p()
    g.malloc(ctypes.byref(dst), 1 << 20)
    for sz, pv in live:
        try:
            g.memcpy(dst, ctypes.c_void_p(pv), sz, 2, None)
            g.device_sync()
        except Exception as e:
            fails += 1
            print("  copy from", hex(pv), "FAIL", str(e)[:120])
    open(path + ".done", "w").write("x")
    print("B fails", fails)


if __name__ == "__main__":
    if len(sys.argv) == 1:
        path = "/tmp/ipc_probe_%d" % os.getpid()
        a = subprocess.Popen([sys.executable, __file__, "A", path])
        b = subprocess.Popen([sys.executable, __file__, "B", path])
        b.wait(timeout=120)
        a.wait(timeout=120)
    else:
        main()
