"""Nodes of a captured HIP graph through the HIP runtime's own C API (ctypes on
libamdhip64.so): node types, and for memset nodes the destination, size and value.  A
diagnostic: TrainStepGraph.node_types(), the graph-replay tests (no memset node may sit in a
captured train step) and tools/graph_reduce_repro.py.  torch: capture with torch.cuda.CUDAGraph(keep_graph=True)
and pass graph.raw_cuda_graph()."""
import contextlib
import ctypes
import gc

import torch

NODE_TYPES = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "graph", 5: "empty",
              6: "wait_event", 7: "event_record", 8: "ext_semas_signal", 9: "ext_semas_wait",
              10: "mem_alloc", 11: "mem_free", 12: "memcpy_from_symbol", 13: "memcpy_to_symbol"}


class _MemsetParams(ctypes.Structure):  # hipMemsetParams (hip_runtime_api.h)
    _fields_ = [("dst", ctypes.c_void_p), ("elementSize", ctypes.c_uint),
                ("height", ctypes.c_size_t), ("pitch", ctypes.c_size_t),
                ("value", ctypes.c_uint), ("width", ctypes.c_size_t)]


_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
    return _hip


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hipError {rc}")


def graph_nodes(raw_graph):
    """[{"type": name, ...}] for every node of the hipGraph_t `raw_graph` (an int)."""
    h = hip()
    g = ctypes.c_void_p(raw_graph)
    n = ctypes.c_size_t(0)
    _check(h.hipGraphGetNodes(g, None, ctypes.byref(n)), "hipGraphGetNodes")
    arr = (ctypes.c_void_p * n.value)()
    _check(h.hipGraphGetNodes(g, arr, ctypes.byref(n)), "hipGraphGetNodes")
    out = []
    for node in arr:
        t = ctypes.c_int(-1)
        _check(h.hipGraphNodeGetType(ctypes.c_void_p(node), ctypes.byref(t)), "hipGraphNodeGetType")
        rec = {"type": NODE_TYPES.get(t.value, str(t.value))}
        if t.value == 2:
            p = _MemsetParams()
            _check(h.hipGraphMemsetNodeGetParams(ctypes.c_void_p(node), ctypes.byref(p)),
                   "hipGraphMemsetNodeGetParams")
            rec.update(dst=p.dst, bytes=p.elementSize * p.width * max(p.height, 1), value=p.value)
        out.append(rec)
    return out


def node_counts(graph):
    """{node type: count} of a torch.cuda.CUDAGraph captured with keep_graph=True."""
    nodes = graph_nodes(graph.raw_cuda_graph())
    out = {}
    for n in nodes:
        out[n["type"]] = out.get(n["type"], 0) + 1
    return out


def read_i32(dev_ptr, count=1):
    """count int32 values at a device address (synchronous hipMemcpy, device -> host)."""
    buf = (ctypes.c_int32 * count)()
    _check(hip().hipMemcpy(buf, ctypes.c_void_p(dev_ptr), ctypes.c_size_t(4 * count), 2),
           "hipMemcpy")
    return list(buf)


@contextlib.contextmanager
def capture(graph, **kw):
    """torch.cuda.graph(graph, **kw) with Python's cyclic garbage collector run BEFORE the
    capture and kept off DURING it.

    torch.cuda.graph does not collect before capture_begin (force_cudagraph_gc is False), so
    reference cycles left by earlier work are collected by whichever allocation crosses the
    collector's threshold -- inside the capture, on the capturing thread.  A dead
    torch.cuda.CUDAGraph in such a cycle is then destroyed inside the capture: ~CUDAGraph's
    device synchronisation (HIPGraph.cpp:324, ROCm builds) returns
    hipErrorStreamCaptureUnsupported, AT_CUDA_CHECK throws in a destructor and std::terminate
    aborts the process -- round 5's 'Fatal Python error: Aborted' under 'Garbage-collecting'
    inside TrainStepGraph._capture, where an earlier test's Trainer <-> TrainStepGraph cycle
    held the graph (tools/capture_finalizer_probe.py)."""
    enabled = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        with torch.cuda.graph(graph, **kw):
            yield
    finally:
        if enabled:
            gc.enable()
