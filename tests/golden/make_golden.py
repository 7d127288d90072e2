"""Regenerate the golden fixtures under tests/golden/ (run in the dev container).

Two sources, both DATA (inputs + expected outputs), no reference source:

1. parquet-mr-written (and Arrow-written) fixture files that the reference's
   own tests hold (parquet-hadoop/src/test/resources/*.parquet,
   parquet-avro/src/test/resources/strings-2.parquet) are copied verbatim.
2. Files written here by pyarrow (Arrow C++ parquet writer, an independent
   third-party writer) with the encodings on the hot path: dictionary
   (RLE_DICTIONARY / PLAIN_DICTIONARY), PLAIN, DELTA_BINARY_PACKED, V1 and V2
   data pages, nulls and nested lists.

For every leaf column chunk the manifest records what the decoder needs
(offsets, physical type, max levels) and the expected dense non-null values as
read back by pyarrow (saved to <file>.npz, so the tests need no pyarrow).
"""
import json
import os
import shutil
import sys

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
REF_FILES = [
    "parquet-hadoop/src/test/resources/test-file-with-no-column-indexes-1.parquet",
    "parquet-hadoop/src/test/resources/test-append_1.parquet",
    "parquet-hadoop/src/test/resources/test-append_2.parquet",
    "parquet-hadoop/src/test/resources/test-empty-row-group_1.parquet",
    "parquet-hadoop/src/test/resources/test-empty-row-group_2.parquet",
    "parquet-hadoop/src/test/resources/test-empty-row-group_3.parquet",
    "parquet-avro/src/test/resources/strings-2.parquet",
]


def leaf_values(arr):
    """Dense non-null leaf values of a (possibly nested) arrow column, in slot order."""
    t = arr.type
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        return leaf_values(pc.list_flatten(arr))
    if pa.types.is_struct(t):
        raise ValueError("struct: select a field first")
    return arr.drop_null()


def field_path_array(table, path):
    """Arrow array of the leaf at dotted `path` with parent nulls/lists preserved."""
    parts = path.split(".")
    arr = table.column(parts[0]).combine_chunks()
    for p in parts[1:]:
        while pa.types.is_list(arr.type):
            arr = pc.list_flatten(arr)
        if pa.types.is_struct(arr.type):
            # propagate struct-level nulls to the child
            child = pc.struct_field(arr, p)
            arr = child
    while pa.types.is_list(arr.type):
        arr = pc.list_flatten(arr)
    return arr


def describe(path_in, name, rg_table_reader):
    pf = pq.ParquetFile(path_in)
    md = pf.metadata
    schema = pf.schema
    chunks = []
    expected = {}
    for rg in range(md.num_row_groups):
        t = pf.read_row_group(rg)
        for c in range(md.num_columns):
            cc = md.row_group(rg).column(c)
            col = schema.column(c)
            path = cc.path_in_schema
            start = cc.dictionary_page_offset if cc.dictionary_page_offset is not None else cc.data_page_offset
            if cc.dictionary_page_offset is not None:
                start = min(cc.dictionary_page_offset, cc.data_page_offset)
            arr = field_path_array(t, path)
            vals = arr.drop_null()
            key = f"rg{rg}_c{c}"
            ptype = col.physical_type
            if ptype == "BYTE_ARRAY":
                b = [bytes(x.as_py() if isinstance(x.as_py(), bytes) else str(x.as_py()).encode()) for x in vals]
                lens = np.array([len(x) for x in b], dtype=np.int64)
                expected[key + "_lens"] = lens
                expected[key + "_bytes"] = np.frombuffer(b"".join(b), dtype=np.uint8) if b else np.zeros(0, np.uint8)
            elif ptype in ("FIXED_LEN_BYTE_ARRAY", "INT96"):
                w = col.length if ptype == "FIXED_LEN_BYTE_ARRAY" else 12
                b = b"".join(bytes(x.as_py()) for x in vals)
                expected[key] = np.frombuffer(b, dtype=np.uint8).reshape(-1, w) if b else np.zeros((0, w), np.uint8)
            elif ptype == "BOOLEAN":
                expected[key] = np.array(vals.to_pylist(), dtype=np.uint8)
            else:
                np_dt = {"INT32": np.int32, "INT64": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}[ptype]
                expected[key] = np.array(vals.to_numpy(zero_copy_only=False), dtype=np_dt) if len(vals) else \
                    np.zeros(0, np_dt)
            chunks.append({"key": key, "row_group": rg, "column": c, "path": path, "physical_type": ptype,
                           "max_def": col.max_definition_level, "max_rep": col.max_repetition_level,
                           "type_length": col.length or 0, "start": start,
                           "length": cc.total_compressed_size, "num_values": cc.num_values,
                           "encodings": list(cc.encodings), "compression": cc.compression,
                           "created_by": md.created_by})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **expected)
    return chunks


def write_arrow_fixtures():
    rng = np.random.default_rng(2024)
    out = []
    n = 30000
    runs = np.minimum(rng.zipf(1.6, size=n), 300)
    ids = np.repeat(rng.integers(0, 500, size=n), runs)[:n]
    d_i64 = rng.integers(-2**62, 2**62, size=500)[ids]
    walk = np.cumsum(rng.integers(-100, 10000, size=n)).astype(np.int64)
    valid = rng.random(n) > 0.1
    t = pa.table({
        "dict_i64": pa.array(d_i64, type=pa.int64()),
        "dict_i32": pa.array((ids * 7 - 1000).astype(np.int32)),
        "dict_f64": pa.array(rng.standard_normal(500)[ids]),
        "opt_dict_i64": pa.array(d_i64, mask=~valid),
        "plain_f32": pa.array(rng.standard_normal(n).astype(np.float32)),
        "opt_plain_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "delta_i64": pa.array(walk),
        "delta_i32": pa.array((walk % 100000).astype(np.int32)),
        "opt_delta_i64": pa.array(walk, mask=~valid),
        "bool": pa.array(rng.random(n) > 0.3),
        "list_i64": pa.array([None if rng.random() < 0.1 else
                              [None if rng.random() < 0.1 else int(x) for x in rng.integers(-50, 50, size=rng.poisson(3))]
                              for _ in range(n // 3)] + [[]] * (n - n // 3)),
    })
    enc = {"delta_i64": "DELTA_BINARY_PACKED", "delta_i32": "DELTA_BINARY_PACKED",
           "opt_delta_i64": "DELTA_BINARY_PACKED", "plain_f32": "PLAIN", "opt_plain_f64": "PLAIN", "bool": "PLAIN"}
    for ver in ("1.0", "2.0"):
        name = f"arrow_encodings_v{ver[0]}"
        path = os.path.join(HERE, name + ".parquet")
        pq.write_table(t, path, data_page_version=ver, compression="NONE",
                       use_dictionary=["dict_i64", "dict_i32", "dict_f64", "opt_dict_i64", "list_i64"],
                       column_encoding=enc, data_page_size=16 * 1024, row_group_size=20000,
                       write_page_index=False)
        out.append(name)
    return out


def write_arrow_binary_fixtures():
    """BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY columns and the remaining value encodings:
    PLAIN and dictionary strings, DELTA_LENGTH_BYTE_ARRAY, DELTA_BYTE_ARRAY (sorted keys with
    shared prefixes), BYTE_STREAM_SPLIT (float/double/int32/int64/FLBA), FLBA dictionary."""
    rng = np.random.default_rng(2025)
    out = []
    n = 8000
    alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
    def rand_str(lo, hi):
        return alpha[rng.integers(0, alpha.size, size=rng.integers(lo, hi + 1))].tobytes().decode()
    words = [rand_str(0, 24) for _ in range(300)]
    runs = np.minimum(rng.zipf(1.5, size=n), 200)
    ids = np.repeat(rng.integers(0, len(words), size=n), runs)[:n]
    valid = rng.random(n) > 0.1
    keys = sorted(f"https://example.org/item/{rng.integers(0, 10**6):07d}/{rand_str(0, 6)}" for _ in range(n))
    fl = [rng.integers(0, 256, size=16, dtype=np.uint8).tobytes() for _ in range(50)]
    t = pa.table({
        "plain_str": pa.array([rand_str(4, 32) for _ in range(n)]),
        "opt_plain_str": pa.array([rand_str(0, 40) if v else None for v in valid]),
        "dict_str": pa.array([words[i] for i in ids]),
        "opt_dict_str": pa.array([words[i] if v else None for i, v in zip(ids, valid)]),
        "dlba_str": pa.array([rand_str(0, 60) for _ in range(n)]),
        "dba_keys": pa.array(keys),
        "opt_dba_str": pa.array([words[i] if v else None for i, v in zip(ids, valid)]),
        "bss_f32": pa.array(rng.standard_normal(n).astype(np.float32)),
        "bss_f64": pa.array(rng.standard_normal(n)),
        "opt_bss_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "bss_i32": pa.array(rng.integers(-2**31, 2**31, size=n).astype(np.int32)),
        "bss_i64": pa.array(rng.integers(-2**40, 2**40, size=n)),
        "bss_flba": pa.array([fl[i % 50] for i in ids], type=pa.binary(16)),
        "dict_flba": pa.array([fl[i % 50] for i in ids], type=pa.binary(16)),
        "plain_flba": pa.array([rng.integers(0, 256, size=5, dtype=np.uint8).tobytes() for _ in range(n)],
                               type=pa.binary(5)),
    })
    enc = {"plain_str": "PLAIN", "opt_plain_str": "PLAIN", "dlba_str": "DELTA_LENGTH_BYTE_ARRAY",
           "dba_keys": "DELTA_BYTE_ARRAY", "opt_dba_str": "DELTA_BYTE_ARRAY", "bss_f32": "BYTE_STREAM_SPLIT",
           "bss_f64": "BYTE_STREAM_SPLIT", "opt_bss_f64": "BYTE_STREAM_SPLIT", "bss_i32": "BYTE_STREAM_SPLIT",
           "bss_i64": "BYTE_STREAM_SPLIT", "bss_flba": "BYTE_STREAM_SPLIT", "plain_flba": "PLAIN"}
    for ver in ("1.0", "2.0"):
        name = f"arrow_binary_v{ver[0]}"
        path = os.path.join(HERE, name + ".parquet")
        pq.write_table(t, path, data_page_version=ver, compression="NONE",
                       use_dictionary=["dict_str", "opt_dict_str", "dict_flba"], column_encoding=enc,
                       data_page_size=16 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def write_arrow_snappy_fixtures():
    """SNAPPY-compressed chunks (the codec parquet-mr writes by default): dictionary, PLAIN,
    DELTA and string columns, optional with nulls, V1 and V2 pages."""
    rng = np.random.default_rng(77)
    n = 12000
    runs = np.minimum(rng.zipf(1.6, size=n), 200)
    ids = np.repeat(rng.integers(0, 300, size=n), runs)[:n]
    valid = rng.random(n) > 0.15
    words = [f"w{i:04d}-{'x' * (i % 17)}" for i in range(300)]
    t = pa.table({
        "dict_i64": pa.array(rng.integers(-2**60, 2**60, size=300)[ids], type=pa.int64()),
        "opt_plain_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "delta_i64": pa.array(np.cumsum(rng.integers(-50, 5000, size=n)).astype(np.int64)),
        "dict_str": pa.array([words[i] for i in ids]),
        "opt_plain_str": pa.array([words[i][: 3 + i % 9] for i in rng.integers(0, 300, size=n)], mask=~valid),
    })
    out = []
    for ver in ("1.0", "2.0"):
        name = f"arrow_snappy_v{ver[0]}"
        pq.write_table(t, os.path.join(HERE, name + ".parquet"), data_page_version=ver, compression="SNAPPY",
                       use_dictionary=["dict_i64", "dict_str"],
                       column_encoding={"opt_plain_f64": "PLAIN", "delta_i64": "DELTA_BINARY_PACKED",
                                        "opt_plain_str": "PLAIN"},
                       data_page_size=8 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def write_arrow_zstd_fixtures():
    """ZSTD-compressed chunks (parquet-mr's ZstandardCodec, level 3 by default): the SNAPPY fixtures'
    table, V1 and V2 pages, so every page kind goes through the device ZSTD decoder."""
    rng = np.random.default_rng(78)
    n = 12000
    runs = np.minimum(rng.zipf(1.6, size=n), 200)
    ids = np.repeat(rng.integers(0, 300, size=n), runs)[:n]
    valid = rng.random(n) > 0.15
    words = [f"w{i:04d}-{'x' * (i % 17)}" for i in range(300)]
    t = pa.table({
        "dict_i64": pa.array(rng.integers(-2**60, 2**60, size=300)[ids], type=pa.int64()),
        "opt_plain_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "delta_i64": pa.array(np.cumsum(rng.integers(-50, 5000, size=n)).astype(np.int64)),
        "dict_str": pa.array([words[i] for i in ids]),
        "opt_plain_str": pa.array([words[i][: 3 + i % 9] for i in rng.integers(0, 300, size=n)], mask=~valid),
        "plain_i32": pa.array(rng.integers(-2**31, 2**31, size=n).astype(np.int32)),
    })
    out = []
    for ver in ("1.0", "2.0"):
        name = f"arrow_zstd_v{ver[0]}"
        pq.write_table(t, os.path.join(HERE, name + ".parquet"), data_page_version=ver, compression="ZSTD",
                       compression_level=3, use_dictionary=["dict_i64", "dict_str"],
                       column_encoding={"opt_plain_f64": "PLAIN", "delta_i64": "DELTA_BINARY_PACKED",
                                        "opt_plain_str": "PLAIN", "plain_i32": "PLAIN"},
                       data_page_size=8 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def write_arrow_lz4_fixtures():
    """LZ4_RAW-compressed chunks (parquet-mr's Lz4RawCodec; pyarrow writes codec LZ4_RAW for
    compression="LZ4"): the ZSTD fixtures' table, V1 and V2 pages, through the device LZ4 decoder."""
    rng = np.random.default_rng(79)
    n = 12000
    runs = np.minimum(rng.zipf(1.6, size=n), 200)
    ids = np.repeat(rng.integers(0, 300, size=n), runs)[:n]
    valid = rng.random(n) > 0.15
    words = [f"w{i:04d}-{'x' * (i % 17)}" for i in range(300)]
    t = pa.table({
        "dict_i64": pa.array(rng.integers(-2**60, 2**60, size=300)[ids], type=pa.int64()),
        "opt_plain_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "delta_i64": pa.array(np.cumsum(rng.integers(-50, 5000, size=n)).astype(np.int64)),
        "dict_str": pa.array([words[i] for i in ids]),
        "opt_plain_str": pa.array([words[i][: 3 + i % 9] for i in rng.integers(0, 300, size=n)], mask=~valid),
        "plain_i64": pa.array(np.cumsum(rng.integers(-100, 1000, size=n)).astype(np.int64)),
    })
    out = []
    for ver in ("1.0", "2.0"):
        name = f"arrow_lz4raw_v{ver[0]}"
        pq.write_table(t, os.path.join(HERE, name + ".parquet"), data_page_version=ver, compression="LZ4",
                       use_dictionary=["dict_i64", "dict_str"],
                       column_encoding={"opt_plain_f64": "PLAIN", "delta_i64": "DELTA_BINARY_PACKED",
                                        "opt_plain_str": "PLAIN", "plain_i64": "PLAIN"},
                       data_page_size=8 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def write_arrow_gzip_fixtures():
    """GZIP-compressed chunks (parquet-mr's GZIP codec: Hadoop GzipCodec, gzip members): the LZ4_RAW
    fixtures' table, V1 and V2 pages, through the device GZIP decoder."""
    rng = np.random.default_rng(80)
    n = 12000
    runs = np.minimum(rng.zipf(1.6, size=n), 200)
    ids = np.repeat(rng.integers(0, 300, size=n), runs)[:n]
    valid = rng.random(n) > 0.15
    words = [f"w{i:04d}-{'x' * (i % 17)}" for i in range(300)]
    t = pa.table({
        "dict_i64": pa.array(rng.integers(-2**60, 2**60, size=300)[ids], type=pa.int64()),
        "opt_plain_f64": pa.array(rng.standard_normal(n), mask=~valid),
        "delta_i64": pa.array(np.cumsum(rng.integers(-50, 5000, size=n)).astype(np.int64)),
        "dict_str": pa.array([words[i] for i in ids]),
        "opt_plain_str": pa.array([words[i][: 3 + i % 9] for i in rng.integers(0, 300, size=n)], mask=~valid),
        "plain_i64": pa.array(np.cumsum(rng.integers(-100, 1000, size=n)).astype(np.int64)),
    })
    out = []
    for ver in ("1.0", "2.0"):
        name = f"arrow_gzip_v{ver[0]}"
        pq.write_table(t, os.path.join(HERE, name + ".parquet"), data_page_version=ver, compression="GZIP",
                       use_dictionary=["dict_i64", "dict_str"],
                       column_encoding={"opt_plain_f64": "PLAIN", "delta_i64": "DELTA_BINARY_PACKED",
                                        "opt_plain_str": "PLAIN", "plain_i64": "PLAIN"},
                       data_page_size=8 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def write_arrow_bool_rle_fixtures():
    """BOOLEAN values with the RLE encoding (4-byte length + width-1 hybrid stream; what
    parquet-mr's V2 writer emits for booleans, DefaultV2ValuesWriterFactory.getBooleanValuesWriter):
    runs, random bits, optional with nulls, inside a list; V1 and V2 pages."""
    rng = np.random.default_rng(91)
    n = 20000
    runs = np.minimum(rng.zipf(1.4, size=n), 3000)
    runbits = np.repeat(rng.random(n) < 0.5, runs)[:n]
    valid = rng.random(n) > 0.2
    t = pa.table({
        "bool_runs": pa.array(runbits),
        "bool_rand": pa.array(rng.random(n) < 0.3),
        "opt_bool": pa.array(rng.random(n) < 0.6, mask=~valid),
        "list_bool": pa.array([None if rng.random() < 0.1 else
                               [None if rng.random() < 0.1 else bool(x) for x in rng.random(rng.poisson(2)) < 0.5]
                               for _ in range(n)]),
    })
    out = []
    for ver in ("1.0", "2.0"):
        name = f"arrow_bool_rle_v{ver[0]}"
        pq.write_table(t, os.path.join(HERE, name + ".parquet"), data_page_version=ver, compression="NONE",
                       use_dictionary=False, column_encoding={c: "RLE" for c in t.column_names},
                       data_page_size=2 * 1024, row_group_size=n, write_page_index=False)
        out.append(name)
    return out


def add_fixtures(writer_fn):
    """Append the fixtures of one writer function to an existing manifest (the others untouched)."""
    with open(os.path.join(HERE, "manifest.json")) as f:
        manifest = json.load(f)
    for name in writer_fn():
        manifest[name] = {"source": "pyarrow " + pa.__version__, "chunks": describe(os.path.join(HERE, name + ".parquet"),
                                                                                   name, None)}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("manifest:", len(manifest), "fixtures")


def main():
    manifest = {}
    for rel in REF_FILES:
        src = os.path.join(REF, rel)
        name = os.path.splitext(os.path.basename(rel))[0]
        dst = os.path.join(HERE, name + ".parquet")
        shutil.copyfile(src, dst)
        manifest[name] = {"source": f"reference:{rel}", "chunks": describe(dst, name, None)}
    for name in (write_arrow_fixtures() + write_arrow_binary_fixtures() + write_arrow_snappy_fixtures() +
                 write_arrow_bool_rle_fixtures() + write_arrow_zstd_fixtures() + write_arrow_lz4_fixtures() +
                 write_arrow_gzip_fixtures()):
        manifest[name] = {"source": "pyarrow " + pa.__version__, "chunks": describe(os.path.join(HERE, name + ".parquet"),
                                                                                   name, None)}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(manifest), "fixtures")


if __name__ == "__main__":
    if "--snappy" in sys.argv:
        sys.exit(add_fixtures(write_arrow_snappy_fixtures))
    if "--zstd" in sys.argv:
        sys.exit(add_fixtures(write_arrow_zstd_fixtures))
    if "--gzip" in sys.argv:
        sys.exit(add_fixtures(write_arrow_gzip_fixtures))
    if "--lz4" in sys.argv:
        sys.exit(add_fixtures(write_arrow_lz4_fixtures))
    if "--bool-rle" in sys.argv:
        sys.exit(add_fixtures(write_arrow_bool_rle_fixtures))
    sys.exit(main())
