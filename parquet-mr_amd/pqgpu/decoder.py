"""Device-side column decoder: the Python face of the C ABI.

`Decoder` owns one pqg_ctx (one HIP stream) per GPU — the analogue of one
ColumnReader per thread in parquet-mr (ColumnReaderBase is not thread-safe).
A `PageBatch` (batch.build_batch, or any caller that lays page bodies out in
one buffer) is uploaded once (`upload`) and decoded into dense device columns:
values of the non-null slots in slot order plus u8 def / rep levels per slot —
the same sequence the reference's ValuesReader / ColumnReader return
(ColumnReaderBase.java:584-676).

torch is used only for device memory and the stream handle.
"""
import ctypes as C
import time

import numpy as np
import torch

from . import abi, batch, native


class DeviceBatch:
    """A PageBatch resident in HBM."""

    def __init__(self, batch, device):
        self.batch = batch
        self.device = device
        self.bytes = torch.from_numpy(batch.data).to(device)
        self.codec_jobs = None  # [(codec, compressed blocks, job table, status, n)] when built by Decoder.upload_chunks

    @property
    def n_bytes(self):
        return int(self.batch.data.size)


class DeviceColumn:
    def __init__(self, physical_type, values, def_levels=None, rep_levels=None, type_length=0, binary_data=None):
        self.physical_type = physical_type
        self.type_length = type_length
        self.values = values          # torch uint8 buffer viewed per type by `typed()` (BYTE_ARRAY: int64 offsets)
        self.def_levels = def_levels
        self.rep_levels = rep_levels
        self.binary_data = binary_data  # BYTE_ARRAY: the values' bytes (offsets index into it)
        self.n_values = 0

    def offsets(self):
        """BYTE_ARRAY: int64 offsets[n_values + 1] (device tensor)."""
        return self.values[: (self.n_values + 1) * 8].view(torch.int64)

    def typed(self):
        dt = {abi.INT32: torch.int32, abi.INT64: torch.int64, abi.FLOAT: torch.float32,
              abi.DOUBLE: torch.float64, abi.BOOLEAN: torch.uint8}.get(self.physical_type)
        w = abi.elem_width(self.physical_type, self.type_length)
        v = self.values[: self.n_values * w]
        return v.view(dt) if dt is not None else v.view(-1, w)

    def numpy(self):
        """Host copy of the decoded values (numpy, the reference's Java array analogue;
        BYTE_ARRAY: a list of bytes, the reference's Binary values)."""
        if self.physical_type == abi.BYTE_ARRAY:
            offs = self.offsets().cpu().numpy()
            data = self.binary_data[: int(offs[-1])].cpu().numpy().tobytes() if offs[-1] > 0 else b""
            return [data[offs[i]:offs[i + 1]] for i in range(self.n_values)]
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

    @property
    def timeout_fallbacks(self):
        """Launches re-run in split mode after a fused-kernel wait timed out (pqg_plan_timeout_fallbacks)."""
        return native.lib().pqg_plan_timeout_fallbacks(self.handle)

    @property
    def plain_fallbacks(self):
        """Launches re-run on the per-value BYTE_ARRAY path because a PLAIN page held bytes after its
        values (pqg_plan_plain_fallbacks)."""
        return native.lib().pqg_plan_plain_fallbacks(self.handle)

    @property
    def null_hint_fallbacks(self):
        """Launches re-run level-first because a V2 header's num_nulls disagreed with the page's
        definition levels (pqg_plan_null_hint_fallbacks)."""
        return native.lib().pqg_plan_null_hint_fallbacks(self.handle)

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

    def set_dispatch(self, key, value):
        """pqg_ctx_set_dispatch: kernel-choice override for plans created afterwards (abi.DISPATCH_*)."""
        native.check(native.lib().pqg_ctx_set_dispatch(self.ctx, int(key), int(value)), what="pqg_ctx_set_dispatch")

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

    _CODEC_FN = {batch.SNAPPY: ("pqg_snappy_decompress", "pqg_snappy_sync", "snappy block"),
                 batch.ZSTD: ("pqg_zstd_decompress", "pqg_zstd_sync", "zstd frame"),
                 batch.LZ4_RAW: ("pqg_lz4_raw_decompress", "pqg_lz4_raw_sync", "lz4_raw block"),
                 batch.GZIP: ("pqg_gzip_decompress", "pqg_gzip_sync", "gzip stream")}

    def upload_chunks(self, chunks):
        """Column chunks whose pages may be SNAPPY-, GZIP-, ZSTD- or LZ4_RAW-compressed -> a DeviceBatch of
        uncompressed pages.

        The batch is laid out for the uncompressed pages (batch.build_batch over placeholders of
        the uncompressed sizes), the compressed blocks are uploaded once, and
        the codec kernels (pqg_snappy / zstd / lz4_raw / gzip_decompress) write every block straight into its page's
        place in the batch on the GPU (ColumnChunkPageReadStore.readPage's decompress step).
        Raises PqgError(CORRUPT / EOF) with the failing block when a block is malformed or its
        length differs from the header."""
        import copy
        placeholders, blocks = [], []   # (codec, payload, ("dict", chunk) | ("page", page index), prefix)
        n_page = 0
        for ch in chunks:
            ph = copy.copy(ch)
            ph.pages = []
            if ch.dict_page is not None and ch.dict_codec != batch.UNCOMPRESSED:
                if ch.dict_codec not in self._CODEC_FN:
                    raise native.PqgError(abi.ERR_UNSUPPORTED, what=f"dictionary page codec {ch.dict_codec}")
                ph.dict_page = bytes(ch.dict_uncompressed_size)
                blocks.append((ch.dict_codec, ch.dict_page, ("dict", len(placeholders)), 0))
            for pg in ch.pages:
                q = copy.copy(pg)
                if pg.codec in self._CODEC_FN:
                    lv = pg.rl_byte_length + pg.dl_byte_length if pg.version == 2 else 0
                    q.body = pg.body[:lv] + bytes(pg.uncompressed_size - lv)
                    blocks.append((pg.codec, pg.body[lv:], ("page", n_page), lv))
                elif pg.codec != batch.UNCOMPRESSED:
                    raise native.PqgError(abi.ERR_UNSUPPORTED, what=f"page codec {pg.codec}")
                ph.pages.append(q)
                n_page += 1
            placeholders.append(ph)
        hb = batch.build_batch(placeholders)
        dbatch = DeviceBatch(hb, self.device)
        if not blocks:
            return dbatch
        col_of_chunk = []
        seen = {}
        for i, ch in enumerate(placeholders):
            seen.setdefault(getattr(ch, "column_index", i), len(seen))
            col_of_chunk.append(seen[getattr(ch, "column_index", i)])
        jobsets = []
        for codec in sorted({b[0] for b in blocks}):
            mine = [b for b in blocks if b[0] == codec]
            src, pos = [], 0
            table = np.zeros(len(mine), dtype=np.dtype([("src_offset", "<u8"), ("dst_offset", "<u8"),
                                                        ("src_size", "<u4"), ("dst_size", "<u4")]))
            for j, (_, payload, (kind, idx), prefix) in enumerate(mine):
                if kind == "dict":
                    dst = int(hb.columns[col_of_chunk[idx]]["dict_offset"])
                    n_out = int(hb.columns[col_of_chunk[idx]]["dict_size"])
                else:
                    dst = int(hb.pages["offset"][idx]) + prefix
                    n_out = int(hb.pages["size"][idx]) - prefix
                table[j] = (pos, dst, len(payload), n_out)
                src.append(payload + bytes((-len(payload)) % 16))
                pos += len(src[-1])
            d_src = torch.from_numpy(np.frombuffer(b"".join(src) + bytes(16), dtype=np.uint8).copy()).to(self.device)
            d_jobs = torch.from_numpy(table.view(np.uint8).copy()).to(self.device)
            d_status = torch.zeros(len(mine), dtype=torch.int32, device=self.device)
            jobsets.append((codec, d_src, d_jobs, d_status, len(mine)))
        torch.cuda.current_stream(self.device).synchronize()  # the uploads above, before the decoder's stream
        dbatch.codec_jobs = jobsets
        self.decompress(dbatch)
        for codec, _, _, d_status, n in jobsets:
            st = abi.Status()
            _, sync, what = self._CODEC_FN[codec]
            rc = getattr(native.lib(), sync)(self.ctx, d_status.data_ptr(), n, C.byref(st))
            native.check(rc, st, what=what)
        return dbatch

    def decompress(self, dbatch):
        """(Re)issue the page decompression of an upload_chunks batch on the decoder's stream
        (asynchronous; the benchmarks time it together with the decode)."""
        for codec, d_src, d_jobs, d_status, n in getattr(dbatch, "codec_jobs", None) or ():
            fn = getattr(native.lib(), self._CODEC_FN[codec][0])
            rc = fn(self.ctx, d_src.data_ptr(), d_src.numel(), dbatch.bytes.data_ptr(), dbatch.n_bytes,
                    d_jobs.data_ptr(), n, d_status.data_ptr())
            native.check(rc, what=self._CODEC_FN[codec][0])

    def zstd_decompress(self, frames, sizes):
        """Raw Zstandard frames (host bytes) -> device tensor of the concatenated outputs (each at a
        16-byte aligned offset) + the offsets, decompressed by pqg_zstd_decompress.
        Returns (out_tensor, offsets, status_codes, status)."""
        src, soff, pos = [], [], 0
        for b in frames:
            soff.append(pos)
            src.append(bytes(b) + bytes((-len(b)) % 16))
            pos += len(src[-1])
        doff = np.concatenate([[0], np.cumsum([(s + 15) // 16 * 16 + 16 for s in sizes])]).astype(np.int64)
        table = np.zeros(len(frames), dtype=np.dtype([("src_offset", "<u8"), ("dst_offset", "<u8"),
                                                      ("src_size", "<u4"), ("dst_size", "<u4")]))
        table["src_offset"], table["dst_offset"] = soff, doff[:-1]
        table["src_size"], table["dst_size"] = [len(b) for b in frames], sizes
        d_src = torch.from_numpy(np.frombuffer(b"".join(src) + bytes(16), dtype=np.uint8).copy()).to(self.device)
        d_dst = torch.zeros(int(doff[-1]) + 16, dtype=torch.uint8, device=self.device)
        d_jobs = torch.from_numpy(table.view(np.uint8).copy()).to(self.device)
        d_status = torch.full((max(len(frames), 1),), -1, dtype=torch.int32, device=self.device)
        torch.cuda.current_stream(self.device).synchronize()
        L = native.lib()
        native.check(L.pqg_zstd_decompress(self.ctx, d_src.data_ptr(), d_src.numel(), d_dst.data_ptr(), d_dst.numel(),
                                           d_jobs.data_ptr(), len(frames), d_status.data_ptr()),
                     what="pqg_zstd_decompress")
        st = abi.Status()
        L.pqg_zstd_sync(self.ctx, d_status.data_ptr(), len(frames), C.byref(st))
        return d_dst, doff, d_status[:len(frames)].cpu().numpy(), st

    def snappy_decompress(self, blocks, sizes, skew=False):
        """Raw Snappy blocks (host bytes) -> device tensor of the concatenated outputs (each at a
        16-byte aligned offset, or with skew=True at offsets of every residue mod 16) + the
        offsets, decompressed by pqg_snappy_decompress. Returns (out_tensor, offsets, status_codes)."""
        return self._block_jobs("pqg_snappy_decompress", "pqg_snappy_sync", blocks, sizes, skew)

    def lz4_raw_decompress(self, blocks, sizes, skew=False):
        """Raw LZ4 blocks (host bytes) -> as snappy_decompress, by pqg_lz4_raw_decompress."""
        return self._block_jobs("pqg_lz4_raw_decompress", "pqg_lz4_raw_sync", blocks, sizes, skew)

    def gzip_decompress(self, blocks, sizes, skew=False):
        """GZIP streams (host bytes) -> as snappy_decompress, by pqg_gzip_decompress."""
        return self._block_jobs("pqg_gzip_decompress", "pqg_gzip_sync", blocks, sizes, skew)

    def _block_jobs(self, fn, fn_sync, blocks, sizes, skew):
        src, soff, pos = [], [], 0
        for b in blocks:
            soff.append(pos)
            src.append(bytes(b) + bytes((-len(b)) % 16))
            pos += len(src[-1])
        doff = np.concatenate([[0], np.cumsum([(s + 15) // 16 * 16 + 16 for s in sizes])]).astype(np.int64)
        if skew:  # block i starts i % 16 bytes into its slot (V2 data sections follow their levels)
            doff[:-1] += np.arange(len(sizes)) % 16
        table = np.zeros(len(blocks), dtype=np.dtype([("src_offset", "<u8"), ("dst_offset", "<u8"),
                                                      ("src_size", "<u4"), ("dst_size", "<u4")]))
        table["src_offset"], table["dst_offset"] = soff, doff[:-1]
        table["src_size"], table["dst_size"] = [len(b) for b in blocks], sizes
        d_src = torch.from_numpy(np.frombuffer(b"".join(src) + bytes(16), dtype=np.uint8).copy()).to(self.device)
        d_dst = torch.zeros(int(doff[-1]) + 16, dtype=torch.uint8, device=self.device)
        d_jobs = torch.from_numpy(table.view(np.uint8).copy()).to(self.device)
        d_status = torch.full((max(len(blocks), 1),), -1, dtype=torch.int32, device=self.device)
        torch.cuda.current_stream(self.device).synchronize()
        L = native.lib()
        native.check(getattr(L, fn)(self.ctx, d_src.data_ptr(), d_src.numel(), d_dst.data_ptr(), d_dst.numel(),
                                    d_jobs.data_ptr(), len(blocks), d_status.data_ptr()), what=fn)
        st = abi.Status()
        getattr(L, fn_sync)(self.ctx, d_status.data_ptr(), len(blocks), C.byref(st))
        return d_dst, doff, d_status[:len(blocks)].cpu().numpy()

    @staticmethod
    def binary_estimate(batch, i):
        """Bytes a BYTE_ARRAY column is first given: its page bytes (PLAIN / DELTA_LENGTH values fit
        in them) + twice its dictionary page; decode() grows it when the device counts more."""
        cd = batch.columns[i]
        pages = batch.pages[batch.pages["column"] == i]
        est = int(pages["size"].sum()) + 2 * int(cd["dict_size"] if cd["dict_offset"] >= 0 else 0) + 64
        if cd["dict_offset"] >= 0 and 0 < cd["dict_num_values"] <= 1 << 16:
            # dictionary column: at most slots x the longest dictionary entry ([u32 length][bytes] each)
            d = batch.data[int(cd["dict_offset"]): int(cd["dict_offset"]) + int(cd["dict_size"])].tobytes()
            pos, longest = 0, 0
            for _ in range(int(cd["dict_num_values"])):
                if pos + 4 > len(d):
                    break
                n = int.from_bytes(d[pos:pos + 4], "little")
                if pos + 4 + n > len(d):  # a corrupt entry (the decode reports it): no size from it
                    break
                longest = max(longest, n)
                pos += 4 + n
            est = max(est, batch.column_slots[i] * longest + 64)
        return est

    def alloc_columns(self, batch):
        cols = []
        for i, cd in enumerate(batch.columns):
            n = batch.column_slots[i]
            w = abi.elem_width(cd["physical_type"], cd["type_length"])
            binary = None
            if cd["physical_type"] == abi.BYTE_ARRAY:
                n_off = n + 1  # offsets[n + 1]
                binary = torch.empty(self.binary_estimate(batch, i), dtype=torch.uint8, device=self.device)
                vals = torch.empty(max(n_off * 8, 16), dtype=torch.uint8, device=self.device)
            else:
                vals = torch.empty(max(n * w, 16), dtype=torch.uint8, device=self.device)
            dl = torch.zeros(max(n, 1), dtype=torch.uint8, device=self.device) if cd["max_def"] > 0 else None
            rl = torch.zeros(max(n, 1), dtype=torch.uint8, device=self.device) if cd["max_rep"] > 0 else None
            if self.poison is not None:
                for t in (vals, dl, rl):
                    if t is not None:
                        t.fill_(self.poison)
            cols.append(DeviceColumn(cd["physical_type"], vals, dl, rl, cd["type_length"], binary))
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
            if cd["physical_type"] == abi.BYTE_ARRAY:
                c.values_capacity = n + 1
                c.binary_data = col.binary_data.data_ptr()
                c.binary_capacity = col.binary_data.numel()
            c.def_levels = col.def_levels.data_ptr() if col.def_levels is not None else None
            c.rep_levels = col.rep_levels.data_ptr() if col.rep_levels is not None else None
            c.levels_capacity = n
        return arr

    # -- decode --------------------------------------------------------------------
    def decode(self, dbatch, cols=None, page_counts=None, check=True):
        """Decode every page of `dbatch` into device columns. Returns (columns, status).
        A BYTE_ARRAY column whose byte buffer turns out short (the status names the bytes it
        needs) is given that many bytes and the batch is decoded again."""
        batch = dbatch.batch
        cols = cols if cols is not None else self.alloc_columns(batch)
        for _ in range(len(batch.columns) + 1):
            rc, st, descs = self._decode_once(dbatch, cols, page_counts)
            if not (rc == abi.ERR_INVALID_ARG and st.page == -1 and st.message.startswith(b"binary capacity")):
                break
            i = int(st.message.split()[3])
            cols[i].binary_data = torch.empty(int(st.value_index) + 64, dtype=torch.uint8, device=self.device)
        for i, col in enumerate(cols):
            col.n_values = int(descs[i].values_written)
        if check:
            native.check(rc, st, "pqg_decode")
        return cols, st

    def _decode_once(self, dbatch, cols, page_counts):
        batch = dbatch.batch
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
        return rc, st, descs

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

    def decode_host(self, batch, binary_capacity=None, prefault=False):
        """File bytes in, host arrays out (pqg_decode_host): the JNI shim's path. BYTE_ARRAY
        columns come back as lists of bytes (plus "offsets"); a short host byte buffer is
        grown to the size the library reports and the call repeated once. prefault=True writes
        the output arrays before the call (a Java `new long[n]` is zeroed, i.e. touched, when it
        is allocated); self.last_native_s = seconds inside the last pqg_decode_host call."""
        caps = {i: binary_capacity or self.binary_estimate(batch, i) for i, cd in enumerate(batch.columns)
                if cd["physical_type"] == abi.BYTE_ARRAY}
        for _ in range(2):
            rc, st, res, counts, need = self._decode_host_once(batch, caps, prefault)
            if not need:
                break
            caps.update(need)
        return rc, st, res, counts

    def _decode_host_once(self, batch, caps, prefault=False):
        descs = (abi.ColumnDesc * max(1, len(batch.columns)))()
        outs = []
        for i, cd in enumerate(batch.columns):
            c = descs[i]
            for k, v in cd.items():
                setattr(c, k, v)
            n = batch.column_slots[i]
            binary = cd["physical_type"] == abi.BYTE_ARRAY
            vals = np.zeros(max(n + 1, 1), dtype=abi.numpy_dtype(cd["physical_type"], cd["type_length"]))
            dl = np.zeros(max(n, 1), dtype=np.uint8)
            rl = np.zeros(max(n, 1), dtype=np.uint8)
            bd = np.zeros(max(caps.get(i, 0), 1), dtype=np.uint8) if binary else None
            if prefault:
                for a in (vals, dl if cd["max_def"] > 0 else None, rl if cd["max_rep"] > 0 else None, bd):
                    if a is not None:
                        a.view(np.uint8)[::4096] = 0
            c.values = vals.ctypes.data
            c.values_capacity = n + 1 if binary else n
            c.def_levels = dl.ctypes.data if cd["max_def"] > 0 else None
            c.rep_levels = rl.ctypes.data if cd["max_rep"] > 0 else None
            c.levels_capacity = n
            if binary:
                c.binary_data = bd.ctypes.data
                c.binary_capacity = caps[i]
            outs.append((vals, dl, rl, bd))
        counts = np.zeros(max(1, batch.n_pages), dtype=np.uint32)
        pages = np.ascontiguousarray(batch.pages)
        st = abi.Status()
        t0 = time.perf_counter()
        rc = native.lib().pqg_decode_host(self.ctx, batch.data.ctypes.data, batch.data.size, C.addressof(descs),
                                          len(batch.columns), pages.ctypes.data if len(pages) else None, len(pages),
                                          counts.ctypes.data, C.byref(st))
        self.last_native_s = time.perf_counter() - t0
        need = {}
        if rc == abi.ERR_INVALID_ARG and st.page == -1 and st.message.startswith(b"binary capacity"):
            need[int(st.message.split()[3])] = int(st.value_index)
        res = []
        for i, cd in enumerate(batch.columns):
            n = int(descs[i].values_written)
            vals, dl, rl, bd = outs[i]
            r = {"values": vals[:n], "n_values": n,
                 "def_levels": dl[:batch.column_slots[i]] if cd["max_def"] > 0 else None,
                 "rep_levels": rl[:batch.column_slots[i]] if cd["max_rep"] > 0 else None}
            if bd is not None:
                offs = vals[:n + 1].copy()
                r["offsets"] = offs
                r["values"] = [bd[offs[k]:offs[k + 1]].tobytes() for k in range(n)] if not need else []
            res.append(r)
        return rc, st, res, counts[:batch.n_pages], need

    def page_errors(self, n_pages):
        """Every page's own first error of the last host / device decode (pqg_page_errors):
        list of (code, phase, index)."""
        pe = (abi.PageError * max(1, n_pages))()
        native.check(native.lib().pqg_page_errors(self.ctx, pe, n_pages), what="pqg_page_errors")
        return [(int(e.code), int(e.phase), int(e.index)) for e in pe[:n_pages]]

    def decode_staged(self, batch):
        """The staged host path (pqg_host_input, pqg_decode_staged, pqg_staged_column): the page
        bytes are written into the library's pinned input, the outputs are read from its pinned
        output. Returns (rc, status, per-column dict like decode_host, page counts);
        self.last_native_s = seconds inside pqg_decode_staged."""
        L = native.lib()
        buf = C.c_void_p()
        native.check(L.pqg_host_input(self.ctx, batch.data.size, C.byref(buf)), what="pqg_host_input")
        C.memmove(buf, batch.data.ctypes.data, batch.data.size)
        descs = (abi.ColumnDesc * max(1, len(batch.columns)))()
        for i, cd in enumerate(batch.columns):
            for k, v in cd.items():
                setattr(descs[i], k, v)
        counts = np.zeros(max(1, batch.n_pages), dtype=np.uint32)
        pages = np.ascontiguousarray(batch.pages)
        st = abi.Status()
        t0 = time.perf_counter()
        rc = L.pqg_decode_staged(self.ctx, batch.data.size, C.addressof(descs), len(batch.columns),
                                 pages.ctypes.data if len(pages) else None, len(pages), counts.ctypes.data, C.byref(st))
        self.last_native_s = time.perf_counter() - t0
        if rc != abi.OK and batch.columns:
            probe = abi.StagedOutput()
            if L.pqg_staged_column(self.ctx, 0, C.byref(probe)) != abi.OK:
                native.check(rc, st, what="pqg_decode_staged")  # no plan was made: the call's own status
        res = []
        for i, cd in enumerate(batch.columns):
            o = abi.StagedOutput()
            native.check(L.pqg_staged_column(self.ctx, i, C.byref(o)), what="pqg_staged_column")
            n, ns = int(o.n_values), int(o.n_slots)
            dt = abi.numpy_dtype(cd["physical_type"], cd["type_length"])
            if descs[i].flags & abi.COLUMN_DICTIONARY_IDS:
                dt = np.dtype(np.uint32)
            binary = cd["physical_type"] == abi.BYTE_ARRAY and dt != np.uint32

            def grab(ptr, count, dtype):
                a = np.empty(count, dtype=dtype)
                if count:
                    L.pqg_copy_out(a.ctypes.data, ptr, a.nbytes)
                return a
            r = {"n_values": n,
                 "def_levels": grab(o.def_levels, ns, np.uint8) if o.def_levels else None,
                 "rep_levels": grab(o.rep_levels, ns, np.uint8) if o.rep_levels else None}
            if binary:
                offs = grab(o.values, n + 1, np.int64)
                data = grab(o.binary, int(o.n_binary), np.uint8) if o.binary else np.zeros(0, np.uint8)
                r["offsets"] = offs
                r["values"] = [data[offs[k]:offs[k + 1]].tobytes() for k in range(n)] if o.binary else []
            else:
                r["values"] = grab(o.values, n, dt)
            res.append(r)
        return rc, st, res, counts[:batch.n_pages]

    # -- record assembly -------------------------------------------------------------
    def assemble(self, path, n_slots, def_levels=None, rep_levels=None):
        """Dremel record assembly of one leaf column (pqg_assemble): `path` = repetitions of the
        schema nodes from the root's child to the leaf; levels = the u8 device tensors decode()
        wrote. Returns {"records": n, "nodes": [{"validity": tensor|None, "offsets": tensor|None,
        "n_entries": n}, ...]} with device tensors (RecordReaderImplementation.read's records in
        columnar form)."""
        depth = len(path)
        nodes = (abi.AssemblyNode * depth)()
        for k, rp in enumerate(path):
            nodes[k].repetition = rp
        L = native.lib()
        n_rec = C.c_uint64(0)
        st = abi.Status()
        dptr = def_levels.data_ptr() if def_levels is not None else None
        rptr = rep_levels.data_ptr() if rep_levels is not None else None
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        # first call: entry counts (capacities 0 -> INVALID_ARG with every n_entries filled in)
        rc = L.pqg_assemble(self.ctx, dptr, rptr, n_slots, C.addressof(nodes), depth, C.byref(n_rec), C.byref(st))
        need_alloc = rc == abi.ERR_INVALID_ARG and st.page == -1 and st.message.startswith(b"assembly output capacity")
        if rc != abi.OK and not need_alloc:
            native.check(rc, st, "pqg_assemble")
        out = []
        counts = [int(nodes[k].n_entries) for k in range(depth)]
        # entries of repetition depth r: records (r = 0), elements of the r-th REPEATED node
        at_depth = [int(n_rec.value)]
        for k, rp in enumerate(path):
            if rp == abi.REPEATED:
                at_depth.append(counts[k])
        keep = []
        r = 0
        for k, rp in enumerate(path):
            v = o = None
            if rp == abi.OPTIONAL:
                v = torch.empty(max(counts[k], 1), dtype=torch.uint8, device=self.device)
                nodes[k].validity = v.data_ptr()
                nodes[k].capacity = counts[k]
            elif rp == abi.REPEATED:
                o = torch.empty(at_depth[r] + 1, dtype=torch.int64, device=self.device)  # one list per enclosing entry
                nodes[k].offsets = o.data_ptr()
                nodes[k].capacity = at_depth[r] + 1
                r += 1
            keep.append((v, o))
        rc = L.pqg_assemble(self.ctx, dptr, rptr, n_slots, C.addressof(nodes), depth, C.byref(n_rec), C.byref(st))
        native.check(rc, st, "pqg_assemble")
        for k in range(depth):
            v, o = keep[k]
            out.append({"validity": v[:counts[k]] if v is not None else None, "offsets": o, "n_entries": counts[k]})
        return {"records": int(n_rec.value), "nodes": out}

    def assemble_schema(self, nodes, leaves):
        """Record assembly of every leaf of a schema (pqg_assemble_schema). nodes: [(parent index or
        -1, repetition)] in depth-first order; leaves: [(node index, def tensor|None, rep tensor|None,
        n_slots)] in schema order. Returns {"records": n, "nodes": [{"validity", "offsets",
        "n_entries"}]} (device tensors; a node's outputs come from the first leaf under it)."""
        arr = (abi.SchemaNode * len(nodes))()
        first_slots = [None] * len(nodes)
        for node, _, _, n in leaves:  # capacity bound: slots of the first leaf under the node (+ 1)
            k = node
            while k >= 0:
                if first_slots[k] is None:
                    first_slots[k] = n
                k = nodes[k][0]
        keep = []
        for k, (parent, rp) in enumerate(nodes):
            arr[k].parent, arr[k].repetition = parent, rp
            cap = (first_slots[k] or 0) + 1
            v = o = None
            if rp == abi.OPTIONAL:
                v = torch.empty(cap, dtype=torch.uint8, device=self.device)
                arr[k].validity = v.data_ptr()
            elif rp == abi.REPEATED:
                o = torch.empty(cap, dtype=torch.int64, device=self.device)
                arr[k].offsets = o.data_ptr()
            arr[k].capacity = cap
            keep.append((v, o))
        lv = (abi.SchemaLeaf * max(1, len(leaves)))()
        for i, (node, dl, rl, n) in enumerate(leaves):
            lv[i].node = node
            lv[i].d_def_levels = dl.data_ptr() if dl is not None else None
            lv[i].d_rep_levels = rl.data_ptr() if rl is not None else None
            lv[i].n_slots = n
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        n_rec = C.c_uint64(0)
        st = abi.Status()
        rc = native.lib().pqg_assemble_schema(self.ctx, C.addressof(arr), len(nodes), C.addressof(lv), len(leaves),
                                              C.byref(n_rec), C.byref(st))
        native.check(rc, st, "pqg_assemble_schema")
        out = []
        for k, (parent, rp) in enumerate(nodes):
            v, o = keep[k]
            cnt = int(arr[k].n_entries)
            enc = None
            if o is not None:  # offsets: one per entry of the enclosing repeated node (or record) + 1
                q = parent
                while q >= 0 and nodes[q][1] != abi.REPEATED:
                    q = nodes[q][0]
                enc = int(n_rec.value) if q < 0 else int(arr[q].n_entries)
            out.append({"validity": v[:cnt] if v is not None else None,
                        "offsets": o[:enc + 1] if o is not None else None, "n_entries": cnt})
        return {"records": int(n_rec.value), "nodes": out}

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

    def router_read_runs(self, bit_width, data, in_offsets, counts):
        """Many ParquetReadRouter.read calls in one round trip (pqg_router_read_runs): run r reads
        counts[r] values at byte in_offsets[r] of `data`; the runs' values back to back."""
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        offs = np.ascontiguousarray(in_offsets, dtype=np.uint64)
        cnts = np.ascontiguousarray(counts, dtype=np.uint32)
        out = np.zeros(max(int(cnts.sum()), 1), dtype=np.int32)
        rc = native.lib().pqg_router_read_runs(self.ctx, bit_width, a.ctypes.data if a.size else None, a.size,
                                               offs.ctypes.data, cnts.ctypes.data, len(cnts), out.ctypes.data)
        native.check(rc, what="pqg_router_read_runs")
        return out[:int(cnts.sum())]

    def router_read_page(self, bit_width, stream, pos, count, out=None):
        """ParquetReadRouter.read through the page cache (pqg_router_read_page): `stream` is the
        caller's whole stream (a uint8 array) positioned at byte `pos`, the run's data start; returns
        the run's `count` values (into `out` when given)."""
        a = stream
        left = a.size - pos
        if out is None:
            out = np.zeros(max(count, 1), dtype=np.int32)
        ptr = a.ctypes.data + pos if left > 0 else None
        rc = native.lib().pqg_router_read_page(self.ctx, bit_width, ptr, left, count, out.ctypes.data)
        native.check(rc, what="pqg_router_read_page")
        return out[:count]

    def router_cache_stats(self):
        """(hits, misses) of pqg_router_read_page on this context."""
        import ctypes as C
        h, m = C.c_uint64(), C.c_uint64()
        native.check(native.lib().pqg_router_cache_stats(self.ctx, C.byref(h), C.byref(m)), what="pqg_router_cache_stats")
        return int(h.value), int(m.value)

    def unpack_runs(self, bit_width, d_in, in_offsets, counts, out_offsets, d_out):
        """Batch of bit-packed runs, all device tensors (pqg_unpack_runs)."""
        rc = native.lib().pqg_unpack_runs(self.ctx, bit_width, d_in.data_ptr(), in_offsets.data_ptr(),
                                          counts.data_ptr(), out_offsets.data_ptr(), d_out.data_ptr(),
                                          int(counts.numel()))
        native.check(rc, what="pqg_unpack_runs")
