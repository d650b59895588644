"""Python face of libkcc.so: the reference's hot-path operations, batched.

Names follow the reference (AshutoshNirkhe/KubernetesClusterCapacity,
src/KubeAPI/ClusterCapacity.go = CC):

  get_pod_cpu_memory_requests_limits  <- getPodCPUMemoryRequestsLimits (CC:255-299)
  total_possible_max_replicas          <- main's node loop (CC:101-140)
  convert_cpu_to_milis                 <- convertCPUToMilis (CC:301-319), batched
  to_bytes                             <- bytefmt.ToBytes (BF:75-105), batched
  get_pod_cpu_memory_requests_limits_keyed  <- CC:255-299 over one cluster-wide pod List

Every call goes through the C-ABI into the gfx950 kernels; nothing is computed here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib

COMM_ID_BYTES = 128  # KCC_COMM_ID_BYTES
P2P_HANDLE_BYTES = 64  # KCC_P2P_HANDLE_BYTES


class KccError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_lib.ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _arr(x, dtype) -> np.ndarray:
    a = np.ascontiguousarray(x, dtype=dtype)
    return a


def _p(a) -> C.c_void_p | None:
    if a is None:
        return None
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(a.ctypes.data or 16)


def _dp(t) -> C.c_void_p | None:
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    return C.c_void_p(t.data_ptr())


@dataclass
class RequestSums:
    """Per-node sums, in the return order of getPodCPUMemoryRequestsLimits (CC:298)
    but as arrays: (cpu limits, cpu requests, memory limits, memory requests)."""
    cpu_limits: np.ndarray | None
    cpu_requests: np.ndarray
    memory_limits: np.ndarray | None
    memory_requests: np.ndarray


class CapacityEngine:
    """One libkcc context (one device, or n_gpus devices with node sharding + RCCL)."""

    def __init__(self, device: int = 0, n_gpus: int = 1, lib_path: str | None = None):
        self._lib = _lib.lib(lib_path)
        h = C.c_void_p()
        rc = self._lib.kcc_create(C.byref(h), device, n_gpus)
        if rc != 0:
            raise KccError(rc, self._lib.kcc_create_error().decode())
        self._h = h
        self.device = device
        self.n_gpus = n_gpus

    # -- lifecycle -------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.kcc_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != 0:
            raise KccError(rc, self._lib.kcc_last_error(self._h).decode())

    def reserve(self, max_nodes: int, max_containers: int, max_specs: int):
        self._check(self._lib.kcc_reserve(self._h, max_nodes, max_containers, max_specs))

    # -- host-array API (synchronous) -----------------------------------------
    def get_pod_cpu_memory_requests_limits(self, node_ptr, cpu_req, mem_req, cpu_lim=None,
                                           mem_lim=None) -> RequestSums:
        """CC:255-299 for every node at once: containers grouped per node (CSR)."""
        node_ptr = _arr(node_ptr, np.int64)
        n = node_ptr.size - 1
        if n < 0:
            raise ValueError("node_ptr must hold n_nodes + 1 offsets")
        cpu_req = _arr(cpu_req, np.uint64)
        mem_req = _arr(mem_req, np.int64)
        lim = cpu_lim is not None or mem_lim is not None
        if lim and (cpu_lim is None or mem_lim is None):
            raise ValueError("pass both cpu_lim and mem_lim, or neither")
        cpu_lim = _arr(cpu_lim, np.uint64) if lim else None
        mem_lim = _arr(mem_lim, np.int64) if lim else None
        nc = cpu_req.size
        if mem_req.size != nc or (lim and (cpu_lim.size != nc or mem_lim.size != nc)):
            raise ValueError("container arrays differ in length")
        used_cpu = np.zeros(max(n, 0), np.uint64)
        used_mem = np.zeros(max(n, 0), np.int64)
        lim_cpu = np.zeros(max(n, 0), np.uint64) if lim else None
        lim_mem = np.zeros(max(n, 0), np.int64) if lim else None
        self._check(self._lib.kcc_reduce_requests(
            self._h, n, nc, _p(node_ptr), _p(cpu_req), _p(mem_req), _p(cpu_lim), _p(mem_lim),
            _p(used_cpu), _p(used_mem), _p(lim_cpu), _p(lim_mem)))
        return RequestSums(lim_cpu, used_cpu, lim_mem, used_mem)

    def total_possible_max_replicas(self, alloc_cpu, alloc_mem, alloc_pods, pod_count,
                                    used_cpu, used_mem, spec_cpu, spec_mem):
        """CC:101-140 for S specs.  Returns (totals int64[S], spec_err int32[S])."""
        a = [_arr(alloc_cpu, np.uint64), _arr(alloc_mem, np.int64), _arr(alloc_pods, np.int64),
             _arr(pod_count, np.int64), _arr(used_cpu, np.uint64), _arr(used_mem, np.int64)]
        n = a[0].size
        if any(x.size != n for x in a):
            raise ValueError("node arrays differ in length")
        sc, sm = _arr(spec_cpu, np.uint64), _arr(spec_mem, np.int64)
        if sc.size != sm.size:
            raise ValueError("spec arrays differ in length")
        totals = np.zeros(sc.size, np.int64)
        err = np.zeros(sc.size, np.int32)
        self._check(self._lib.kcc_fit(self._h, n, *[_p(x) for x in a], sc.size, _p(sc), _p(sm),
                                      _p(totals), _p(err)))
        return totals, err

    def capacity(self, node_ptr, cpu_req, mem_req, alloc_cpu, alloc_mem, alloc_pods, pod_count,
                 spec_cpu, spec_mem):
        """Fused (a)+(b) on host arrays.  Returns (totals, spec_err)."""
        node_ptr = _arr(node_ptr, np.int64)
        n = node_ptr.size - 1
        cpu_req, mem_req = _arr(cpu_req, np.uint64), _arr(mem_req, np.int64)
        a = [_arr(alloc_cpu, np.uint64), _arr(alloc_mem, np.int64), _arr(alloc_pods, np.int64),
             _arr(pod_count, np.int64)]
        if any(x.size != n for x in a):
            raise ValueError("node arrays differ in length")
        if cpu_req.size != mem_req.size:
            raise ValueError("container arrays differ in length")
        sc, sm = _arr(spec_cpu, np.uint64), _arr(spec_mem, np.int64)
        totals = np.zeros(sc.size, np.int64)
        err = np.zeros(sc.size, np.int32)
        self._check(self._lib.kcc_capacity(
            self._h, n, cpu_req.size, _p(node_ptr), _p(cpu_req), _p(mem_req),
            *[_p(x) for x in a], sc.size, _p(sc), _p(sm), _p(totals), _p(err)))
        return totals, err

    # -- list-order containers ---------------------------------
    def get_pod_cpu_memory_requests_limits_keyed(self, n_keys, key, cpu_req, mem_req,
                                                 cpu_lim=None, mem_lim=None) -> RequestSums:
        """CC:255-299 for every row at once from containers in list order: key[i] is the
        row of container i's node (<0 or >= n_keys: not on a listed row)."""
        key = _key32(key)
        cpu_req, mem_req = _arr(cpu_req, np.uint64), _arr(mem_req, np.int64)
        lim = cpu_lim is not None or mem_lim is not None
        if lim and (cpu_lim is None or mem_lim is None):
            raise ValueError("pass both cpu_lim and mem_lim, or neither")
        cpu_lim = _arr(cpu_lim, np.uint64) if lim else None
        mem_lim = _arr(mem_lim, np.int64) if lim else None
        nc = key.size
        if cpu_req.size != nc or mem_req.size != nc or (lim and (cpu_lim.size != nc or
                                                                 mem_lim.size != nc)):
            raise ValueError("container arrays differ in length")
        used_cpu, used_mem = np.zeros(n_keys, np.uint64), np.zeros(n_keys, np.int64)
        lim_cpu = np.zeros(n_keys, np.uint64) if lim else None
        lim_mem = np.zeros(n_keys, np.int64) if lim else None
        self._check(self._lib.kcc_reduce_requests_keyed(
            self._h, n_keys, nc, _p(key), _p(cpu_req), _p(mem_req), _p(cpu_lim), _p(mem_lim),
            _p(used_cpu), _p(used_mem), _p(lim_cpu), _p(lim_mem)))
        return RequestSums(lim_cpu, used_cpu, lim_mem, used_mem)

    def count_by_key(self, n_keys, key):
        """len(pods) per row (CC:106, CC:135) from the pods' row keys."""
        key = _key32(key)
        count = np.zeros(n_keys, np.int64)
        self._check(self._lib.kcc_count_by_key(self._h, n_keys, key.size, _p(key), _p(count)))
        return count

    def reduce_requests_keyed_async(self, n_keys, key, cpu_req, mem_req, used_cpu, used_mem,
                                    stream=None):
        self._check(self._lib.kcc_reduce_requests_keyed_async(
            self._h, n_keys, key.numel(), _dp(key), _dp(cpu_req), _dp(mem_req), None, None,
            _dp(used_cpu), _dp(used_mem), None, None, _stream(stream)))

    def pod_requests_async(self, pod_ptr, cpu_req, mem_req, pod_cpu, pod_mem, init_ptr=None,
                           init_cpu=None, init_mem=None, restartable=None, ovh_cpu=None,
                           ovh_mem=None, stream=None):
        """Device form of pod_requests (torch tensors; SURVEY §8f row 4, opt-in)."""
        n_init = 0 if init_cpu is None else init_cpu.numel()
        self._check(self._lib.kcc_pod_requests_async(
            self._h, pod_ptr.numel() - 1, cpu_req.numel(), n_init, _dp(pod_ptr), _dp(cpu_req),
            _dp(mem_req), _dp(init_ptr), _dp(init_cpu), _dp(init_mem), _dp(restartable),
            _dp(ovh_cpu), _dp(ovh_mem), _dp(pod_cpu), _dp(pod_mem), _stream(stream)))

    # -- quantity strings -------------------------------------
    def _parse(self, fn, strings, dtype):
        if isinstance(strings, tuple):
            buf, off = strings
        else:
            from .quantity import pack_strings
            buf, off = pack_strings(strings)
        buf = _arr(buf, np.uint8)
        off = _arr(off, np.int64)
        n = off.size - 1
        if n < 0:
            raise ValueError("offsets must hold n + 1 entries")
        out = np.zeros(n, dtype)
        st = np.zeros(n, np.int8)
        self._check(fn(self._h, n, _p(buf), buf.size, _p(off), _p(out), _p(st)))
        return out, st

    def convert_cpu_to_milis(self, strings):
        """convertCPUToMilis (CC:301-319) over a batch: `strings` is a sequence of str or
        a packed (bytes uint8, offsets int64) pair.  Returns (uint64 values, int8
        status: 1 ok, 0 where the reference prints an error and uses 0)."""
        return self._parse(self._lib.kcc_parse_cpu_millis, strings, np.uint64)

    def to_bytes(self, strings):
        """bytefmt.ToBytes (BF:75-105) over a batch.  Returns (int64 values, int8
        status: 1 ok, 0 error (value 0), -1 outside the device's exact ParseFloat
        domain — see include/kcc.h)."""
        return self._parse(self._lib.kcc_parse_bytes, strings, np.int64)

    def max_replicas_per_row(self, alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu,
                             used_mem, spec_cpu: int, spec_mem: int):
        """CC:119-137 per node row for one spec ("Max replicas" of the verbose report).
        Returns (q int64[N], row_err int32[N]: 1 where Go would panic at that row)."""
        a = [_arr(alloc_cpu, np.uint64), _arr(alloc_mem, np.int64), _arr(alloc_pods, np.int64),
             _arr(pod_count, np.int64), _arr(used_cpu, np.uint64), _arr(used_mem, np.int64)]
        n = a[0].size
        if any(x.size != n for x in a):
            raise ValueError("node arrays differ in length")
        q = np.zeros(n, np.int64)
        err = np.zeros(n, np.int32)
        self._check(self._lib.kcc_fit_rows(self._h, n, *[_p(x) for x in a],
                                           int(spec_cpu) % (1 << 64), int(spec_mem), _p(q),
                                           _p(err)))
        return q, err

    @staticmethod
    def _pod_args(pod_ptr, cpu_req, mem_req, init_ptr, init_cpu, init_mem, restartable,
                  ovh_cpu, ovh_mem):
        pp = _arr(pod_ptr, np.int64)
        if pp.size < 1:
            raise ValueError("pod_ptr needs n_pods + 1 entries")
        n_pods = pp.size - 1
        cr, mr = _arr(cpu_req, np.uint64), _arr(mem_req, np.int64)
        if cr.size != mr.size:
            raise ValueError("container arrays differ in length")
        ip = ic = im = rs = None
        n_init = 0
        if init_ptr is not None:
            ip, ic, im = _arr(init_ptr, np.int64), _arr(init_cpu, np.uint64), _arr(init_mem, np.int64)
            if ip.size != n_pods + 1 or ic.size != im.size:
                raise ValueError("init arrays do not match pod_ptr")
            n_init = ic.size
            if restartable is not None:
                rs = _arr(restartable, np.uint8)
                if rs.size != n_init:
                    raise ValueError("restartable differs in length from the init arrays")
        elif restartable is not None or init_cpu is not None or init_mem is not None:
            raise ValueError("init container arrays without init_ptr")
        oc = None if ovh_cpu is None else _arr(ovh_cpu, np.uint64)
        om = None if ovh_mem is None else _arr(ovh_mem, np.int64)
        for o in (oc, om):
            if o is not None and o.size != n_pods:
                raise ValueError("overhead arrays need one entry per pod")
        return n_pods, cr.size, n_init, [pp, cr, mr, ip, ic, im, rs, oc, om]

    def pod_requests(self, pod_ptr, cpu_req, mem_req, init_ptr=None, init_cpu=None,
                     init_mem=None, restartable=None, ovh_cpu=None, ovh_mem=None):
        """OPT-IN scheduler request model (NOT the reference, which sums
        app containers only, CC:276-294): per pod max(app sum, init max incl. sidecars) +
        overhead — see include/kcc.h.  Returns (uint64 cpu[P], int64 mem[P])."""
        n_pods, n_cont, n_init, a = self._pod_args(pod_ptr, cpu_req, mem_req, init_ptr,
                                                   init_cpu, init_mem, restartable, ovh_cpu,
                                                   ovh_mem)
        pc, pm = np.zeros(n_pods, np.uint64), np.zeros(n_pods, np.int64)
        self._check(self._lib.kcc_pod_requests(self._h, n_pods, n_cont, n_init,
                                               *[_p(x) for x in a], _p(pc), _p(pm)))
        return pc, pm

    def reduce_requests_pods(self, node_pod_ptr, pod_ptr, cpu_req, mem_req, init_ptr=None,
                             init_cpu=None, init_mem=None, restartable=None, ovh_cpu=None,
                             ovh_mem=None):
        """Per-node sums of the opt-in pod requests (pods grouped by node, CSR
        node_pod_ptr[N+1]): the used_cpu / used_mem kcc_fit takes."""
        npp = _arr(node_pod_ptr, np.int64)
        if npp.size < 1:
            raise ValueError("node_pod_ptr needs n_nodes + 1 entries")
        n_nodes = npp.size - 1
        n_pods, n_cont, n_init, a = self._pod_args(pod_ptr, cpu_req, mem_req, init_ptr,
                                                   init_cpu, init_mem, restartable, ovh_cpu,
                                                   ovh_mem)
        uc, um = np.zeros(n_nodes, np.uint64), np.zeros(n_nodes, np.int64)
        self._check(self._lib.kcc_reduce_requests_pods(self._h, n_nodes, n_pods, n_cont, n_init,
                                                       _p(npp), *[_p(x) for x in a], _p(uc),
                                                       _p(um)))
        return uc, um

    def quantity_value(self, strings):
        """resource.Quantity.Value() of ParseQuantity (CC:285-286, parity unpinned: see
        include/kcc.h) over a batch.  Returns (int64 values, int8 status)."""
        return self._parse(self._lib.kcc_parse_quantity, strings, np.int64)

    def last_slow_fraction(self) -> float:
        return float(self._lib.kcc_last_slow_fraction(self._h))

    # -- device API (torch tensors, enqueue on `stream`) -------------------------
    def reduce_requests_async(self, node_ptr, cpu_req, mem_req, used_cpu, used_mem,
                              cpu_lim=None, mem_lim=None, lim_cpu=None, lim_mem=None,
                              stream=None):
        n = node_ptr.numel() - 1
        self._check(self._lib.kcc_reduce_requests_async(
            self._h, n, cpu_req.numel(), _dp(node_ptr), _dp(cpu_req), _dp(mem_req),
            _dp(cpu_lim), _dp(mem_lim), _dp(used_cpu), _dp(used_mem), _dp(lim_cpu),
            _dp(lim_mem), _stream(stream)))

    def fit_prepare_async(self, alloc_cpu, alloc_mem, alloc_pods, pod_count, used_cpu, used_mem,
                          spec_cpu, spec_mem, partial, stream=None):
        self._check(self._lib.kcc_fit_prepare_async(
            self._h, alloc_cpu.numel(), _dp(alloc_cpu), _dp(alloc_mem), _dp(alloc_pods),
            _dp(pod_count), _dp(used_cpu), _dp(used_mem), spec_cpu.numel(), _dp(spec_cpu),
            _dp(spec_mem), _dp(partial), _stream(stream)))

    def fit_run_async(self, n_nodes, n_specs, partial, stream=None):
        self._check(self._lib.kcc_fit_run_async(self._h, n_nodes, n_specs, _dp(partial),
                                                _stream(stream)))

    def fit_finalize_async(self, n_specs, partial, totals, spec_err, stream=None):
        self._check(self._lib.kcc_fit_finalize_async(self._h, n_specs, _dp(partial),
                                                     _dp(totals), _dp(spec_err),
                                                     _stream(stream)))

    def capacity_partial_async(self, h_node_ptr, node_ptr, cpu_req, mem_req, alloc_cpu,
                               alloc_mem, alloc_pods, pod_count, used_cpu, used_mem, spec_cpu,
                               spec_mem, partial, n_chunks=0, stream=None):
        """Pipelined reduce + fit partial (kcc_capacity_partial_async): h_node_ptr is the
        host copy (numpy int64) of node_ptr, used only to place the chunk boundaries."""
        h = None if h_node_ptr is None else np.ascontiguousarray(h_node_ptr, np.int64)
        if h is not None and h.size != node_ptr.numel():
            raise ValueError("h_node_ptr and node_ptr differ in length")
        self._check(self._lib.kcc_capacity_partial_async(
            self._h, node_ptr.numel() - 1, cpu_req.numel(), _p(h), _dp(node_ptr), _dp(cpu_req),
            _dp(mem_req), _dp(alloc_cpu), _dp(alloc_mem), _dp(alloc_pods), _dp(pod_count),
            _dp(used_cpu), _dp(used_mem), spec_cpu.numel(), _dp(spec_cpu), _dp(spec_mem),
            _dp(partial), int(n_chunks), _stream(stream)))

    def capacity_async(self, h_node_ptr, node_ptr, cpu_req, mem_req, alloc_cpu, alloc_mem,
                       alloc_pods, pod_count, used_cpu, used_mem, spec_cpu, spec_mem, totals,
                       spec_err, stream=None):
        """The whole one-device step (kcc_capacity_async): reduce + fit + clamp correction
        with the finalize fused into the last launch -> totals (int64) / spec_err (int32)."""
        h = None if h_node_ptr is None else np.ascontiguousarray(h_node_ptr, np.int64)
        self._check(self._lib.kcc_capacity_async(
            self._h, node_ptr.numel() - 1, cpu_req.numel(), _p(h), _dp(node_ptr), _dp(cpu_req),
            _dp(mem_req), _dp(alloc_cpu), _dp(alloc_mem), _dp(alloc_pods), _dp(pod_count),
            _dp(used_cpu), _dp(used_mem), spec_cpu.numel(), _dp(spec_cpu), _dp(spec_mem),
            _dp(totals), _dp(spec_err), _stream(stream)))

    def parse_cpu_millis_async(self, buf, off, out, status, stream=None):
        self._check(self._lib.kcc_parse_cpu_millis_async(
            self._h, off.numel() - 1, _dp(buf), buf.numel(), _dp(off), _dp(out), _dp(status),
            _stream(stream)))

    def parse_bytes_async(self, buf, off, out, status, stream=None):
        self._check(self._lib.kcc_parse_bytes_async(
            self._h, off.numel() - 1, _dp(buf), buf.numel(), _dp(off), _dp(out), _dp(status),
            _stream(stream)))

    def parse_quantity_async(self, buf, off, out, status, stream=None):
        self._check(self._lib.kcc_parse_quantity_async(
            self._h, off.numel() - 1, _dp(buf), buf.numel(), _dp(off), _dp(out), _dp(status),
            _stream(stream)))

    # -- node sharding ------------------------------------------------
    def set_node_shards(self, n_shards: int):
        """Host-array entry points: cut the nodes into this many contiguous shards
        (round-robin over the context's devices; 0 = one per device)."""
        self._check(self._lib.kcc_set_node_shards(self._h, int(n_shards)))

    @staticmethod
    def comm_unique_id() -> bytes:
        """Rank 0 of a one-process-per-GPU run: the RCCL id every rank passes to
        comm_init (opaque bytes, distributed by the caller)."""
        buf = C.create_string_buffer(COMM_ID_BYTES)
        rc = _lib.lib().kcc_comm_unique_id(C.cast(buf, C.c_void_p))  # (release build)
        if rc != 0:
            raise KccError(rc, "ncclGetUniqueId failed")
        return buf.raw

    def comm_init(self, uid: bytes, n_ranks: int, rank: int):
        """Join the ranks' RCCL communicator (collective: blocks until every rank joined)."""
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"the id holds {COMM_ID_BYTES} bytes")
        buf = C.create_string_buffer(uid, COMM_ID_BYTES)
        self._check(self._lib.kcc_comm_init(self._h, C.cast(buf, C.c_void_p), n_ranks, rank))

    def allreduce_partial_async(self, n_specs, partial, stream=None):
        """RCCL all-reduce (sum, int64) of the 2*S partial vector, on `stream`."""
        self._check(self._lib.kcc_allreduce_partial_async(self._h, n_specs, _dp(partial),
                                                          _stream(stream)))

    def p2p_export(self, n_ranks: int, max_specs: int) -> bytes:
        """One-shot xGMI exchange, setup step 1: allocate this rank's mailbox and return
        its IPC handle (opaque bytes every rank must receive)."""
        buf = C.create_string_buffer(P2P_HANDLE_BYTES)
        self._check(self._lib.kcc_p2p_export(self._h, int(n_ranks), int(max_specs),
                                             C.cast(buf, C.c_void_p)))
        return buf.raw

    def p2p_open(self, rank: int, handles):
        """Setup step 2: map every peer's mailbox (handles: every rank's export, by rank)."""
        blob = b"".join(handles)
        if len(blob) != P2P_HANDLE_BYTES * len(handles):
            raise ValueError(f"each handle holds {P2P_HANDLE_BYTES} bytes")
        buf = C.create_string_buffer(blob, len(blob))
        self._check(self._lib.kcc_p2p_open(self._h, int(rank), C.cast(buf, C.c_void_p)))

    def exchange_finalize_async(self, n_specs, partial, totals, spec_err, stream=None):
        """Each step: push this rank's partial to every peer's mailbox, wait for theirs,
        sum and finalize (replaces allreduce_partial_async + fit_finalize_async)."""
        self._check(self._lib.kcc_exchange_finalize_async(self._h, n_specs, _dp(partial),
                                                          _dp(totals), _dp(spec_err),
                                                          _stream(stream)))

    def p2p_faults(self) -> int:
        """Flag waits of the exchange that gave up (0 on a healthy run)."""
        v = C.c_int64()
        self._check(self._lib.kcc_p2p_faults(self._h, C.byref(v)))
        return v.value

    def profile_enable(self, on: bool = True):
        self._check(self._lib.kcc_profile_enable(self._h, 1 if on else 0))

    def profile_read(self):
        """(reduce_ms_total, reduce_launches, fit_ms_total, fit_launches) of the pipelined
        calls since profile_enable (synchronises)."""
        rm, rn, fm, fn = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        self._check(self._lib.kcc_profile_read(self._h, C.byref(rm), C.byref(rn), C.byref(fm),
                                               C.byref(fn)))
        return rm.value, rn.value, fm.value, fn.value

    def set_fit_dense(self, dense: bool):
        """Stream every node row through the fit (diagnostic); default: only the rows
        that can add to its fast sum."""
        self._check(self._lib.kcc_set_fit_dense(self._h, 1 if dense else 0))

    def set_clamp_in_fit(self, mode: int):
        """-1: the pod-slot clamp inside the fit on small shards (default), 0: always the
        clamp correction launch, 1: inside the fit whenever specs <= 4096."""
        self._check(self._lib.kcc_set_clamp_in_fit(self._h, int(mode)))

    def clamp_in_fit_used(self) -> bool:
        """Whether the last capacity call applied the clamp inside the fit."""
        v = C.c_int()
        self._check(self._lib.kcc_clamp_in_fit_used(self._h, C.byref(v)))
        return bool(v.value)

    def fit_stream_rows(self) -> int:
        """Node rows (padded to groups of 8) the last fit streamed."""
        v = C.c_int64()
        self._check(self._lib.kcc_fit_stream_rows(self._h, C.byref(v)))
        return v.value

    def reduce_faults(self) -> int:
        """Look-back waits of the segmented reduce that gave up (0 on a healthy device)."""
        v = C.c_int64()
        self._check(self._lib.kcc_reduce_faults(self._h, C.byref(v)))
        return v.value

    def clear_faults(self):
        """Reset the device fault words and the reduce's look-back records."""
        self._check(self._lib.kcc_clear_faults(self._h))

    def fit_slow_pairs(self):
        a, b = C.c_int64(), C.c_int64()
        self._check(self._lib.kcc_fit_slow_pairs(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value


def _key32(key) -> np.ndarray:
    """Row keys as int32 (the C-ABI's type); wider keys must fit, never wrap silently."""
    k = np.asarray(key)
    if k.dtype != np.int32 and k.size and (k.max() > np.iinfo(np.int32).max or
                                           k.min() < np.iinfo(np.int32).min):
        raise ValueError("row keys must fit int32")
    return np.ascontiguousarray(k, np.int32)


def _stream(stream):
    if stream is None:
        return None
    h = getattr(stream, "cuda_stream", stream)
    return C.c_void_p(int(h)) if h else None


def verdict(totals, replicas):
    """CC:144: `totalPossibleMaxReplicas >= replicas`, per spec."""
    return np.asarray(totals, np.int64) >= np.asarray(replicas, np.int64)
