"""KernelSpanEvents: HIP timing events recorded by event-record nodes added
to a captured hipGraph (bench.py's kernel-span timing in round 6 until the
stamp kernels replaced it: a graph holding these nodes launched slower from
the host, tools/lab/launch_probe.py).  Kept for the lab probes."""


class KernelSpanEvents:
    """Two HIP timing events recorded by EVENT-RECORD NODES inside the timed
    hipGraphs: after capture (torch.cuda.CUDAGraph(keep_graph=True)) a node
    recording `head` is added before the graph's root nodes and one recording
    `tail` after its leaves (hipGraphAddEventRecordNode /
    hipGraphAddDependencies on raw_cuda_graph()), then the graph is
    instantiated.  Recorded in the first and the last timed graph they bracket
    the step kernels only; the host's graph submission before the first kernel
    is outside.  torch refuses external events on ROCm, so the
    HIP runtime torch itself loaded is called through ctypes."""

    def __init__(self):
        import ctypes
        import torch
        torch.cuda.init()
        path = None
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64.so" in line:
                    path = line.split()[-1]
                    break
        if path is None:
            raise RuntimeError("libamdhip64.so is not mapped in this process")
        self.path = path
        self.hip = ctypes.CDLL(path)
        self.c = ctypes
        self.head, self.tail = ctypes.c_void_p(), ctypes.c_void_p()
        for ev in (self.head, self.tail):
            self._check(self.hip.hipEventCreate(ctypes.byref(ev)), "hipEventCreate")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: hipError {rc}")

    def _nodes(self, fn, *lead):
        c = self.c
        n = c.c_size_t(0)
        self._check(fn(*lead, None, c.byref(n)), fn.__name__)
        arr = (c.c_void_p * max(1, n.value))()
        self._check(fn(*lead, arr, c.byref(n)), fn.__name__)
        return [c.c_void_p(arr[i]) for i in range(n.value)]

    def add_nodes(self, graph, head: bool, tail: bool) -> None:
        """Event-record nodes into a captured, not yet instantiated graph."""
        c, hip = self.c, self.hip
        g = c.c_void_p(graph.raw_cuda_graph())
        if tail:
            leaves = [nd for nd in self._nodes(hip.hipGraphGetNodes, g)
                      if not self._nodes(hip.hipGraphNodeGetDependentNodes, nd)]
            deps = (c.c_void_p * len(leaves))(*[nd.value for nd in leaves])
            node = c.c_void_p()
            self._check(hip.hipGraphAddEventRecordNode(c.byref(node), g, deps, c.c_size_t(len(leaves)), self.tail),
                        "hipGraphAddEventRecordNode(tail)")
        if head:
            roots = self._nodes(hip.hipGraphGetRootNodes, g)
            node = c.c_void_p()
            self._check(hip.hipGraphAddEventRecordNode(c.byref(node), g, None, c.c_size_t(0), self.head),
                        "hipGraphAddEventRecordNode(head)")
            for r in roots:
                self._check(hip.hipGraphAddDependencies(g, c.byref(node), c.byref(r), c.c_size_t(1)),
                            "hipGraphAddDependencies")

    def record(self, which: str, stream) -> None:
        """An ordinary record on the stream (the eager path)."""
        ev = self.head if which == "head" else self.tail
        self._check(self.hip.hipEventRecord(ev, self.c.c_void_p(stream.cuda_stream)), "hipEventRecord")

    def elapsed_ms(self) -> float:
        ms = self.c.c_float(0.0)
        self._check(self.hip.hipEventSynchronize(self.tail), "hipEventSynchronize")
        self._check(self.hip.hipEventElapsedTime(self.c.byref(ms), self.head, self.tail), "hipEventElapsedTime")
        return float(ms.value)

    def close(self):
        for ev in (self.head, self.tail):
            self.hip.hipEventDestroy(ev)
