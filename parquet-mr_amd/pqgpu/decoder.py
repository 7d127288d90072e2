"""Device-side column decoder: the Python face of the C ABI.

`Decoder` owns one pqg_ctx (one HIP stream) per GPU — the analogue of one
ColumnReader per thread in parquet-mr (ColumnReaderBase is not thread-safe).
A `PageBatch` (writer.build_batch, or any caller that lays page bodies out in
one buffer) is uploaded once (`upload`) and decoded into dense device columns:
values of the non-null slots in slot order plus u8 def / rep levels per slot —
the same sequence the reference's ValuesReader / ColumnReader return
(ColumnReaderBase.java:584-676).

torch is used only for device memory and the stream handle.
"""
import ctypes as C

import numpy as np
import torch

from . import abi, native


class DeviceBatch:
    """A PageBatch resident in HBM."""

    def __init__(self, batch, device):
        self.batch = batch
        self.device = device
        self.bytes = torch.from_numpy(batch.data).to(device)

    @property
    def n_bytes(self):
        return int(self.batch.data.size)


class DeviceColumn:
    def __init__(self, physical_type, values, def_levels=None, rep_levels=None, type_length=0):
        self.physical_type = physical_type
        self.type_length = type_length
        self.values = values          # torch uint8 buffer viewed per type by `typed()`
        self.def_levels = def_levels
        self.rep_levels = rep_levels
        self.n_values = 0

    def typed(self):
        dt = {abi.INT32: torch.int32, abi.INT64: torch.int64, abi.FLOAT: torch.float32,
              abi.DOUBLE: torch.float64, abi.BOOLEAN: torch.uint8}.get(self.physical_type)
        w = abi.elem_width(self.physical_type, self.type_length)
        v = self.values[: self.n_values * w]
        return v.view(dt) if dt is not None else v.view(-1, w)

    def numpy(self):
        """Host copy of the decoded values (numpy, the reference's Java array analogue)."""
        w = abi.elem_width(self.physical_type, self.type_length)
        raw = self.values[: self.n_values * w].cpu().numpy()
        return raw.view(abi.numpy_dtype(self.physical_type, self.type_length))


class Plan:
    """A prepared decode of one DeviceBatch (pqg_plan): launch() re-runs it."""

    def __init__(self, decoder, handle, columns, descs, keep):
        self.decoder = decoder
        self.handle = handle
        self.columns = columns
        self._descs = descs
        self._keep = keep

    def launch(self):
        native.check(native.lib().pqg_plan_launch(self.handle), what="pqg_plan_launch")

    @property
    def kernel_count(self):
        return native.lib().pqg_plan_kernel_count(self.handle)

    def sync(self):
        st = abi.Status()
        rc = native.lib().pqg_sync(self.decoder.ctx, C.byref(st))
        return rc, st

    def close(self):
        if self.handle:
            native.lib().pqg_plan_destroy(self.handle)
            self.handle = None


class Decoder:
    def __init__(self, device=0, stream=None, poison=None):
        """poison: byte value written over freshly allocated output columns (tests use it so an
        element the kernels never write, or write twice with different values, cannot pass by
        reusing memory that already holds the right answer)."""
        self.poison = poison
        L = native.lib()
        if L.pqg_device_count() <= 0:
            raise native.PqgError(abi.ERR_NO_DEVICE, what="no HIP device")
        self.device = torch.device("cuda", device)
        torch.cuda.set_device(self.device)
        if stream is None:
            # a dedicated stream: the default stream's handle is 0, which the C ABI reads as
            # "create your own", and events must be recorded on the stream the kernels run on
            stream = torch.cuda.Stream(self.device)
        self.stream = stream
        h = C.c_void_p()
        native.check(L.pqg_ctx_create(device, C.c_void_p(stream.cuda_stream), C.byref(h)), what="pqg_ctx_create")
        self.ctx = h

    def close(self):
        if self.ctx:
            native.lib().pqg_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- buffers -----------------------------------------------------------------
    def upload(self, batch):
        return DeviceBatch(batch, self.device)

    def alloc_columns(self, batch):
        cols = []
        for i, cd in enumerate(batch.columns):
            n = batch.column_slots[i]
            w = abi.elem_width(cd["physical_type"], cd["type_length"])
            vals = torch.empty(max(n * w, 16), dtype=torch.uint8, device=self.device)
            dl = torch.zeros(max(n, 1), dtype=torch.uint8, device=self.device) if cd["max_def"] > 0 else None
            rl = torch.zeros(max(n, 1), dtype=torch.uint8, device=self.device) if cd["max_rep"] > 0 else None
            if self.poison is not None:
                for t in (vals, dl, rl):
                    if t is not None:
                        t.fill_(self.poison)
            cols.append(DeviceColumn(cd["physical_type"], vals, dl, rl, cd["type_length"]))
        return cols

    def _descs(self, batch, cols):
        arr = (abi.ColumnDesc * max(1, len(batch.columns)))()
        for i, cd in enumerate(batch.columns):
            c = arr[i]
            for k, v in cd.items():
                setattr(c, k, v)
            col = cols[i]
            n = batch.column_slots[i]
            c.values = col.values.data_ptr()
            c.values_capacity = n
            c.def_levels = col.def_levels.data_ptr() if col.def_levels is not None else None
            c.rep_levels = col.rep_levels.data_ptr() if col.rep_levels is not None else None
            c.levels_capacity = n
        return arr

    # -- decode --------------------------------------------------------------------
    def decode(self, dbatch, cols=None, page_counts=None, check=True):
        """Decode every page of `dbatch` into device columns. Returns (columns, status)."""
        batch = dbatch.batch
        cols = cols if cols is not None else self.alloc_columns(batch)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))  # uploads / allocations first
        descs = self._descs(batch, cols)
        pages = np.ascontiguousarray(batch.pages)
        st = abi.Status()
        counts_ptr = page_counts.data_ptr() if page_counts is not None else None
        L = native.lib()
        rc = L.pqg_decode(self.ctx, dbatch.bytes.data_ptr(), dbatch.n_bytes, C.addressof(descs), len(batch.columns),
                          pages.ctypes.data if len(pages) else None, len(pages), counts_ptr, C.byref(st))
        if rc == abi.OK:
            rc = L.pqg_sync(self.ctx, C.byref(st))
        for i, col in enumerate(cols):
            col.n_values = int(descs[i].values_written)
        if check:
            native.check(rc, st, "pqg_decode")
        return cols, st

    def plan(self, dbatch, cols=None):
        batch = dbatch.batch
        cols = cols if cols is not None else self.alloc_columns(batch)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        descs = self._descs(batch, cols)
        pages = np.ascontiguousarray(batch.pages)
        st = abi.Status()
        h = C.c_void_p()
        rc = native.lib().pqg_plan_create(self.ctx, dbatch.bytes.data_ptr(), dbatch.n_bytes, C.addressof(descs),
                                          len(batch.columns), pages.ctypes.data if len(pages) else None, len(pages),
                                          C.byref(h), C.byref(st))
        native.check(rc, st, "pqg_plan_create")
        for i, col in enumerate(cols):
            col.n_values = batch.column_values[i]
        return Plan(self, h, cols, descs, (pages, dbatch))

    def decode_host(self, batch):
        """File bytes in, host arrays out (pqg_decode_host): the JNI shim's path."""
        descs = (abi.ColumnDesc * max(1, len(batch.columns)))()
        outs = []
        for i, cd in enumerate(batch.columns):
            c = descs[i]
            for k, v in cd.items():
                setattr(c, k, v)
            n = batch.column_slots[i]
            vals = np.zeros(max(n, 1), dtype=abi.numpy_dtype(cd["physical_type"], cd["type_length"]))
            dl = np.zeros(max(n, 1), dtype=np.uint8)
            rl = np.zeros(max(n, 1), dtype=np.uint8)
            c.values = vals.ctypes.data
            c.values_capacity = n
            c.def_levels = dl.ctypes.data if cd["max_def"] > 0 else None
            c.rep_levels = rl.ctypes.data if cd["max_rep"] > 0 else None
            c.levels_capacity = n
            outs.append((vals, dl, rl))
        counts = np.zeros(max(1, batch.n_pages), dtype=np.uint32)
        pages = np.ascontiguousarray(batch.pages)
        st = abi.Status()
        rc = native.lib().pqg_decode_host(self.ctx, batch.data.ctypes.data, batch.data.size, C.addressof(descs),
                                          len(batch.columns), pages.ctypes.data if len(pages) else None, len(pages),
                                          counts.ctypes.data, C.byref(st))
        res = []
        for i, cd in enumerate(batch.columns):
            n = int(descs[i].values_written)
            vals, dl, rl = outs[i]
            res.append({"values": vals[:n], "n_values": n,
                        "def_levels": dl[:batch.column_slots[i]] if cd["max_def"] > 0 else None,
                        "rep_levels": rl[:batch.column_slots[i]] if cd["max_rep"] > 0 else None})
        return rc, st, res, counts[:batch.n_pages]

    # -- ParquetReadRouter ---------------------------------------------------------
    def router_read(self, bit_width, data, count):
        """ParquetReadRouter.read(bitWidth, in, currentCount, int[]) on the GPU."""
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        out = np.zeros(max(count, 1), dtype=np.int32)
        rc = native.lib().pqg_router_read(self.ctx, bit_width, a.ctypes.data if a.size else None, a.size, count,
                                          out.ctypes.data)
        native.check(rc, what="pqg_router_read")
        return out[:count]

    def unpack_runs(self, bit_width, d_in, in_offsets, counts, out_offsets, d_out):
        """Batch of bit-packed runs, all device tensors (pqg_unpack_runs)."""
        rc = native.lib().pqg_unpack_runs(self.ctx, bit_width, d_in.data_ptr(), in_offsets.data_ptr(),
                                          counts.data_ptr(), out_offsets.data_ptr(), d_out.data_ptr(),
                                          int(counts.numel()))
        native.check(rc, what="pqg_unpack_runs")
