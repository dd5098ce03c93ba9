"""Combining queue for concurrent per-tensor plugin calls.

OpenFL reaches the codec one tensor per call, from several threads at once:
the gRPC server's ThreadPoolExecutor (transport/grpc/aggregator_server.py:305)
runs one handler per collaborator RPC, and the aggregator decompresses outside
its lock (component/aggregator/aggregator.py:643-646).  Each call is one GPU
round trip (H2D, launches, D2H, one synchronisation), so concurrent calls pay
those round trips one after the other on the device's queue.

Combiner merges them (flat combining): a caller appends its request; if no
call is being served, it becomes the leader, takes every pending request (its
own included) and runs them as ONE batch (one H2D, one launch sequence, one
D2H, one synchronisation), hands every caller its own result, then passes the
leadership to the oldest waiting caller, if any.  A caller alone (no
concurrency) runs a batch of one: the per-tensor path it had before.
Results equal the per-call ones: the batch functions are the pipelines'
forward_batch / backward_batch internals, whose bytes are identical to
per-tensor calls (tests/test_gpu_parity.py::test_pipeline_batch_equals_per_tensor),
and anything order-dependent (the np.random draw of the Eden seed) is taken
by the caller at entry, in call order, before it joins the queue.
"""
import threading


class _Req:
    __slots__ = ("item", "result", "error", "done", "lead")

    def __init__(self, item):
        self.item = item
        self.result = None
        self.error = None
        self.done = threading.Event()
        self.lead = False


class Combiner:
    """run_batch(list of items) -> list of results, same order."""

    def __init__(self, run_batch, max_items=256):
        self.run_batch = run_batch
        self.max_items = int(max_items)
        self._lock = threading.Lock()
        self._pending = []
        self._active = False
        self.batches = 0          # statistics (tests, benches)
        self.items = 0

    def call(self, item):
        req = _Req(item)
        with self._lock:
            self._pending.append(req)
            lead = not self._active
            if lead:
                self._active = True
        if not lead:
            req.done.wait()
            if not req.lead:      # served by a leader
                if req.error is not None:
                    raise req.error
                return req.result
        # leader: serve batches until this request is done, then hand over
        while True:
            with self._lock:
                batch = self._pending[:self.max_items]
                del self._pending[:len(batch)]
            if batch:
                try:
                    res = self.run_batch([r.item for r in batch])
                    if len(res) != len(batch):
                        raise RuntimeError("combiner: batch returned a wrong number of results")
                    for r, x in zip(batch, res):
                        r.result = x
                except BaseException as e:  # every caller of the batch sees the failure
                    for r in batch:
                        r.error = e
                self.batches += 1
                self.items += len(batch)
                for r in batch:
                    if r is not req:
                        r.done.set()
            if req.result is not None or req.error is not None or not batch:
                break
        with self._lock:
            if self._pending:     # the oldest waiting caller leads next
                nxt = self._pending[0]
                nxt.lead = True
                nxt.done.set()
            else:
                self._active = False
        if req.error is not None:
            raise req.error
        return req.result
