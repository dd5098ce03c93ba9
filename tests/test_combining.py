"""openfl_amd.combining.Combiner: concurrent per-tensor calls merged into
batches (flat combining with leader hand-off).  CPU only: the batch function
here is plain Python; the GPU test (test_gpu_parity.py::
test_concurrent_plugin_calls_combine) runs the Eden pipeline through it."""
import threading
import time

import pytest

from openfl_amd.combining import Combiner


def test_single_caller_runs_batches_of_one():
    seen = []
    c = Combiner(lambda items: seen.append(list(items)) or [x * 2 for x in items])
    assert [c.call(i) for i in range(5)] == [0, 2, 4, 6, 8]
    assert seen == [[0], [1], [2], [3], [4]] and c.batches == 5 and c.items == 5


def test_concurrent_callers_get_their_own_results_in_fewer_batches():
    gate = threading.Event()
    sizes = []

    def run(items):
        gate.wait(5)            # the first leader holds the device while the others queue
        sizes.append(len(items))
        time.sleep(0.002)
        return [("r", x) for x in items]
    c = Combiner(run)
    out = {}

    def worker(k):
        for j in range(20):
            out[(k, j)] = c.call((k, j))
    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    time.sleep(0.05)
    gate.set()
    for t in th:
        t.join(10)
    assert all(not t.is_alive() for t in th)
    assert out == {(k, j): ("r", (k, j)) for k in range(8) for j in range(20)}
    assert c.items == 160 and c.batches < 160 and max(sizes) > 1


def test_batch_failure_reaches_every_caller_of_the_batch():
    def run(items):
        if any(x < 0 for x in items):
            raise ValueError("bad item")
        return items
    c = Combiner(run)
    with pytest.raises(ValueError):
        c.call(-1)
    assert c.call(3) == 3      # the combiner is usable afterwards


def test_leadership_passes_on():
    """A leader serves batches until its own request is done, then hands the
    queue to the oldest waiting caller: nobody waits forever and no request
    is served twice."""
    served = []
    lock = threading.Lock()

    def run(items):
        with lock:
            served.extend(items)
        time.sleep(0.001)
        return items
    c = Combiner(run, max_items=3)
    th = [threading.Thread(target=lambda k=k: [c.call((k, j)) for j in range(30)]) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join(20)
    assert all(not t.is_alive() for t in th)
    assert sorted(served) == sorted((k, j) for k in range(6) for j in range(30))
    assert c.items == 180 and not c._active and not c._pending
