"""ORACLE — TEST INFRASTRUCTURE ONLY: record assembly of one leaf column.

A pure-Python restatement (small cases only) of parquet-mr's Dremel record assembly
automaton, RecordReaderImplementation (parquet-column/.../io/RecordReaderImplementation.java),
for a projection onto ONE leaf column, plus a converter from the automaton's converter events
to the columnar (Arrow-style) form the GPU kernels produce (pqg_assemble, include/pqgpu.h).

Automaton (single leaf, i.e. one State):
  * nextLevel[r] (levelToClose, :284-306): r == 0 -> 0 (end of record closes every group);
    r > 0 -> the leaf is the last leaf under its level-r repeated ancestor (isLast), so the
    groups are closed down to that ancestor: getParent(r).getFieldPath().length - 1 (:296-298).
  * definitionLevelToDepth[d] (:314-324): index of the deepest group on the path whose
    definition level is <= d (-1 for none).
  * read() (:409-446): per slot open groups up to definitionLevelToDepth[d], emit the value when
    d >= maxDefinitionLevel, then close groups down to nextLevel[next slot's r]; r == 0 ends
    the record.

Only tests/ import this module.
"""

REQUIRED, OPTIONAL, REPEATED = 0, 1, 2


def levels_of(path):
    """Cumulative (repetition, definition) level of every node (ColumnIO.getRepetitionLevel /
    getDefinitionLevel): REPEATED adds one to both, OPTIONAL one to the definition level."""
    r = d = 0
    out = []
    for rep in path:
        if rep == REPEATED:
            r += 1
            d += 1
        elif rep == OPTIONAL:
            d += 1
        out.append((r, d))
    return out


def fsm_events(path, names, rep_levels, def_levels, values):
    """Converter events of RecordReaderImplementation.read for the leaf `path` (node repetitions,
    root's child .. leaf) over one column's slots. values: the dense non-null values.
    Events: ("startMessage",), ("start", k), ("end", k), ("value", v), ("endMessage",);
    k indexes the group nodes path[0 .. L-2]."""
    L = len(path)
    lv = levels_of(path)
    max_r, max_d = lv[-1]
    # nextLevel[r] (levelToClose)
    next_level = [0] * (max_r + 1)
    for r in range(1, max_r + 1):
        parent = max(k for k in range(L) if path[k] == REPEATED and lv[k][0] == r)  # getParent(r)
        next_level[r] = parent  # fieldPath length of node `parent` (0-based index + 1) - 1
    # definitionLevelToDepth[d]
    d2depth = []
    for d in range(max_d + 1):
        depth = 0
        while depth < L - 1 and d >= lv[depth][1]:
            depth += 1
        d2depth.append(depth - 1)
    ev = []
    n = len(def_levels)
    vi = 0
    i = 0
    while i < n:
        ev.append(("startMessage",))
        cur = 0
        while True:
            d = int(def_levels[i])
            depth = d2depth[d]
            while cur <= depth:
                ev.append(("start", cur))
                cur += 1
            if d >= max_d:
                ev.append(("value", values[vi]))
                vi += 1
            i += 1
            next_r = 0 if (max_r == 0 or i >= n) else int(rep_levels[i])
            nxt = next_level[next_r]
            while cur > nxt:
                ev.append(("end", cur - 1))
                cur -= 1
            if next_r == 0:
                break
        ev.append(("endMessage",))
    return ev


def event_strings(path, names, ev):
    """Events in TestColumnIO's string form (ExpectationValidatingConverter), e.g.
    'Name.Language.start()', 'Name.Url.addBinary(http://A)', 'DocId.addLong(10)'."""
    out = []
    leaf = ".".join(names)
    for e in ev:
        if e[0] == "startMessage":
            out.append("startMessage()")
        elif e[0] == "endMessage":
            out.append("endMessage()")
        elif e[0] in ("start", "end"):
            out.append(".".join(names[:e[1] + 1]) + f".{e[0]}()")
        else:
            v = e[1]
            out.append(f"{leaf}.addBinary({v.decode()})" if isinstance(v, bytes) else f"{leaf}.addLong({v})")
    return out


def columnar(path, ev):
    """Columnar form of an event stream (what pqg_assemble returns):
      records: number of records;
      per node k: OPTIONAL -> validity list (one per entry of its repetition depth),
                  REPEATED -> offsets list (one per entry of the enclosing depth, + final count).
    Entries of repetition depth r are the records (r = 0) or the elements of the r-th repeated
    node; a non-repeated node has one entry per entry of its depth."""
    L = len(path)
    lv = levels_of(path)
    depth_of = [lv[k][0] for k in range(L)]          # repetition depth of node k's entries
    max_r = lv[-1][0]
    validity = {k: [] for k in range(L) if path[k] == OPTIONAL}
    offsets = {k: [] for k in range(L) if path[k] == REPEATED}
    count = {k: 0 for k in offsets}
    pending = {}                                      # optional node -> present in the open entry
    open_depth = -1                                   # deepest depth with an open entry

    def close_to(r):  # close open entries of depth >= r
        nonlocal open_depth
        while open_depth >= r:
            for k in validity:
                if depth_of[k] == open_depth and k in pending:
                    validity[k].append(pending.pop(k))
            open_depth -= 1

    def open_entry(r):
        nonlocal open_depth
        close_to(r)
        open_depth = r
        for k in validity:
            if depth_of[k] == r:
                pending[k] = 0
        for k in offsets:
            if depth_of[k] == r + 1:
                offsets[k].append(count[k])

    records = 0
    for e in ev:
        if e[0] == "startMessage":
            records += 1
            open_entry(0)
        elif e[0] == "start":
            k = e[1]
            if path[k] == REPEATED:
                count[k] += 1
                open_entry(depth_of[k])
            elif path[k] == OPTIONAL:
                pending[k] = 1
        elif e[0] == "value":
            k = L - 1
            if path[k] == REPEATED:
                count[k] += 1
                open_entry(depth_of[k])
            elif path[k] == OPTIONAL:
                pending[k] = 1
        elif e[0] == "endMessage":
            pass
    close_to(0)
    for k in offsets:
        offsets[k].append(count[k])
    del max_r
    return {"records": records, "validity": validity, "offsets": offsets}
