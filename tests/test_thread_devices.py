"""Thread -> device mapping of multi-GPU plugin settings (codec.ThreadDevices):
SURVEY 8(e) -- unchanged callers reach several GPUs through the gRPC
server's concurrent worker threads (aggregator_server.py:305), so a plugin
naming several devices binds each calling thread to one, round-robin."""
import threading

import pytest

from openfl_amd.codec import PerThreadDevice, ThreadDevices


def test_round_robin_and_sticky():
    td = ThreadDevices(3)
    got = [None] * 12
    barrier = threading.Barrier(12)

    def work(i):
        barrier.wait()
        a = td.slot()
        got[i] = (a, td.slot(), td.slot())  # sticky within a thread

    th = [threading.Thread(target=work, args=(i,)) for i in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(a == b == c for a, b, c in got)
    firsts = sorted(a for a, _, _ in got)
    assert firsts == sorted([0, 1, 2] * 4)  # 12 threads spread 4 per device


def test_main_thread_slot_stable():
    td = ThreadDevices(2)
    assert td.slot() == td.slot() == 0


def test_invalid():
    with pytest.raises(ValueError):
        ThreadDevices(0)


def test_shared_mapping_follows():
    class T(PerThreadDevice):
        def __init__(self, devs, share=None):
            if share is None:
                self.devices, self._thread_devices = list(devs), ThreadDevices(len(devs))
            else:
                self._init_devices(None, share)

    a = T(["d0", "d1"])
    b = T(None, share=a)
    seen = []

    def work():
        seen.append((a.device, b.device))

    th = [threading.Thread(target=work) for _ in range(4)]
    for t in th:
        t.start()
        t.join()
    assert all(x == y for x, y in seen)
    assert sorted(x for x, _ in seen) == ["d0", "d0", "d1", "d1"]


def test_numa_cpulist_parsing():
    """openfl_amd.numa reads sysfs cpulists ("0-3,8,10-11") into CPU sets."""
    from openfl_amd import numa
    assert numa._cpulist("0-3,8,10-11") == {0, 1, 2, 3, 8, 10, 11}
    assert numa._cpulist("64-127,192-255") == set(range(64, 128)) | set(range(192, 256))
    assert numa._cpulist("") == set() and numa._cpulist(None) == set()
