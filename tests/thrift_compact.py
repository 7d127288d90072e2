"""Thrift compact-protocol PageHeader writer for tests (parquet.thrift PageHeader / DataPageHeader /
DictionaryPageHeader / DataPageHeaderV2, TCompactProtocol): builds raw column-chunk bytes (headers +
bodies) the way a parquet writer lays them out, so framing and the C harness can be fed file bytes
for synthetic chunks. Test infrastructure only."""
import zlib



def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(n):
    return _varint((n << 1) ^ (n >> 63))


def _struct(fields):
    """fields: [(fid, type, payload bytes)] in increasing fid order -> compact struct bytes."""
    out, last = bytearray(), 0
    for fid, t, payload in fields:
        d = fid - last
        out += bytes([(d << 4) | t]) if 0 < d <= 15 else bytes([t]) + _zz(fid)
        out += payload
        last = fid
    return bytes(out + b"\x00")


def page_header(ptype, size, num_values, enc=0, crc=None, v2=None, extra_field=False, usize=None, is_compressed=False):
    """usize: uncompressed_page_size (default = size); is_compressed: the V2 header's flag."""
    f = [(1, 5, _zz(ptype)), (2, 5, _zz(size if usize is None else usize)), (3, 5, _zz(size))]
    if crc is not None:
        f.append((4, 5, _zz(crc - (1 << 32) if crc >= 1 << 31 else crc)))
    if ptype == 0:
        f.append((5, 12, _struct([(1, 5, _zz(num_values)), (2, 5, _zz(enc)), (3, 5, _zz(3)), (4, 5, _zz(3))])))
    elif ptype == 2:
        f.append((7, 12, _struct([(1, 5, _zz(num_values)), (2, 5, _zz(enc))])))
    elif ptype == 3:
        rl, dl = v2
        f.append((8, 12, _struct([(1, 5, _zz(num_values)), (2, 5, _zz(0)), (3, 5, _zz(num_values)),
                                  (4, 5, _zz(enc)), (5, 5, _zz(dl)), (6, 5, _zz(rl)),
                                  (7, 1 if is_compressed else 2, b"")])))
    if extra_field:  # an unknown field id 20 (binary) the reader must skip
        f.append((20, 8, _varint(3) + b"xyz"))
    return _struct(f)


def page_header_of(pg, crc=None, usize=None, is_compressed=False):
    """PageHeader of a writer.Page (uncompressed unless the caller says otherwise: usize =
    uncompressed_page_size to claim, is_compressed = the V2 flag)."""
    if pg.version == 2:
        return page_header(3, len(pg.body), pg.num_values, enc=pg.encoding, crc=crc,
                           v2=(pg.rl_byte_length, pg.dl_byte_length), usize=usize, is_compressed=is_compressed)
    f = [(1, 5, _zz(0)), (2, 5, _zz(len(pg.body) if usize is None else usize)), (3, 5, _zz(len(pg.body)))]
    if crc is not None:
        f.append((4, 5, _zz(crc - (1 << 32) if crc >= 1 << 31 else crc)))
    f.append((5, 12, _struct([(1, 5, _zz(pg.num_values)), (2, 5, _zz(pg.encoding)), (3, 5, _zz(pg.dl_encoding)),
                              (4, 5, _zz(pg.rl_encoding))])))
    return _struct(f)


def chunk_bytes(ch, with_crc=True, dict_num_values=None, is_compressed=False):
    """Raw bytes of an uncompressed writer.ColumnChunk: [dictionary page] data pages, each header
    followed by its body (with page CRCs, as parquet-mr writes them by default). is_compressed: the
    V2 headers' flag (the bodies stay as they are)."""
    out = bytearray()
    if ch.dict_page is not None:
        crc = zlib.crc32(ch.dict_page) if with_crc else None
        n = ch.dict_num_values if dict_num_values is None else dict_num_values
        out += page_header(2, len(ch.dict_page), n, enc=ch.dict_encoding, crc=crc) + ch.dict_page
    for pg in ch.pages:
        out += page_header_of(pg, zlib.crc32(pg.body) if with_crc else None, is_compressed=is_compressed) + pg.body
    return bytes(out)
