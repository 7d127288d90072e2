"""ORACLE — TEST INFRASTRUCTURE ONLY: record assembly (one leaf column, and every leaf of a schema).

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


# ---- all leaves of a schema (the automaton proper) -------------------------------------------------------

class Node:
    """A schema node: name, repetition, children (a leaf has none)."""

    def __init__(self, name, repetition, children=()):
        self.name, self.repetition, self.children = name, repetition, list(children)


def schema_leaves(roots):
    """Leaves in schema order (MessageColumnIO.getLeaves) with their node chains (root's child .. leaf)."""
    out = []

    def walk(n, chain):
        chain = chain + [n]
        if not n.children:
            out.append(chain)
        for c in n.children:
            walk(c, chain)
    for r in roots:
        walk(r, [])
    return out


def fsm_events_multi(roots, columns):
    """Converter events of RecordReaderImplementation.read over every leaf of the schema
    (RecordReaderImplementation.java:253-330 builds the automaton, :409-446 runs it).
    columns: per leaf (schema order) a tuple (rep_levels, def_levels, dense values).
    Events: ("startMessage",), ("start", name path), ("end", name path), ("value", leaf path, v),
    ("endMessage",)."""
    leaves = schema_leaves(roots)
    n_leaves = len(leaves)
    lv = []                          # per leaf: (r, d) of every node on its path
    for chain in leaves:
        lv.append(levels_of([n.repetition for n in chain]))

    def parent_idx(i, r):            # ColumnIO.getParent(r): index on the path (-1: the message root)
        chain, levels = leaves[i], lv[i]
        for k in range(len(chain) - 1, -1, -1):
            if levels[k][0] == r and chain[k].repetition == REPEATED:
                return k
            if k == 0 or levels[k - 1][1] < r:   # getParent().getDefinitionLevel() >= r fails
                break
        if r == 0:
            return -1
        raise ValueError(f"no parent({r})")

    def subtree_leaves(i, k):         # leaf indices under node k of leaf i's path (-1: all)
        if k < 0:
            return list(range(n_leaves))
        node = leaves[i][k]
        return [j for j in range(n_leaves) if len(leaves[j]) > k and leaves[j][k] is node]

    def is_first(i, r):
        return subtree_leaves(i, parent_idx(i, r))[0] == i

    def is_last(i, r):
        return subtree_leaves(i, parent_idx(i, r))[-1] == i

    def common(i, j):                 # getCommonParentLevel(fieldPath_i, fieldPath_j)
        a, b = leaves[i], leaves[j]
        k = 0
        while k < min(len(a), len(b)) and a[k] is b[k]:
            k += 1
        return k

    first_for_level = [0] * 256
    next_col, level_to_close, d2depth = [], [], []
    for i in range(n_leaves):
        max_r, max_d = lv[i][-1]
        nc, ltc = [], []
        for r in range(max_r + 1):
            if is_first(i, r):
                first_for_level[r] = i
            if r == 0:
                nxt = i + 1
            elif is_last(i, r):
                nxt = first_for_level[r]
            else:
                nxt = i + 1
            if nxt == n_leaves:
                close = 0
            elif is_last(i, r):
                # parent.getFieldPath().length - 1: the parent's index on the path (r > 0 here)
                close = parent_idx(i, r)
            else:
                close = common(i, nxt)
            nc.append(nxt)
            ltc.append(close)
        next_col.append(nc)
        level_to_close.append(ltc)
        # definitionLevelToDepth (:324-333)
        L = len(leaves[i])
        dd, depth = [], 0
        for d in range(max_d + 1):
            while depth < L - 1 and d >= lv[i][depth][1]:
                depth += 1
            dd.append(depth - 1)
        d2depth.append(dd)
    pos = [[0, 0] for _ in range(n_leaves)]   # per leaf: next slot, next value
    ev = []
    n0 = len(columns[0][1]) if n_leaves else 0
    while n_leaves and pos[0][0] < n0:
        ev.append(("startMessage",))
        cur, i = 0, 0
        while i is not None:
            rl, dl, vals = columns[i]
            chain = leaves[i]
            names = [n.name for n in chain]
            s = pos[i][0]
            d = int(dl[s])
            depth = d2depth[i][d]
            while cur <= depth:
                ev.append(("start", ".".join(names[:cur + 1])))
                cur += 1
            if d >= lv[i][-1][1]:
                ev.append(("value", ".".join(names), vals[pos[i][1]]))
                pos[i][1] += 1
            pos[i][0] = s + 1
            max_r = lv[i][-1][0]
            nr = 0 if (max_r == 0 or s + 1 >= len(dl)) else int(rl[s + 1])
            nxt = level_to_close[i][nr]
            while cur > nxt:
                ev.append(("end", ".".join(names[:cur])))
                cur -= 1
            ni = next_col[i][nr]
            i = None if ni == n_leaves else ni
        ev.append(("endMessage",))
    return ev


def event_strings_multi(ev):
    """TestColumnIO's string form of fsm_events_multi events."""
    out = []
    for e in ev:
        if e[0] == "startMessage":
            out.append("startMessage()")
        elif e[0] == "endMessage":
            out.append("endMessage()")
        elif e[0] in ("start", "end"):
            out.append(f"{e[1]}.{e[0]}()")
        else:
            v = e[2]
            out.append(f"{e[1]}.addBinary({v.decode()})" if isinstance(v, bytes) else f"{e[1]}.addLong({v})")
    return out


def columnar_multi(roots, ev):
    """Columnar form of a whole-schema event stream (what pqg_assemble_schema returns), keyed by
    the node's dotted name: OPTIONAL -> validity (one per instance of its nearest REPEATED
    ancestor-or-self, or per record), REPEATED -> offsets (one per instance of the enclosing
    repeated node or record, + the final count). 'records' -> number of records."""
    info = {}                                   # path -> (repetition, owner, enclosing owner, is_leaf)

    def walk(n, prefix, owner):
        path = prefix + n.name
        own = path if n.repetition == REPEATED else owner
        info[path] = (n.repetition, own, owner, not n.children)
        for c in n.children:
            walk(c, path + ".", own)
    for r in roots:
        walk(r, "", "")
    validity = {p: [] for p, v in info.items() if v[0] == OPTIONAL}
    offsets = {p: [] for p, v in info.items() if v[0] == REPEATED}
    count = {p: 0 for p in offsets}
    records = 0

    def new_instance(o):                      # an instance of owner o ("" = a record) opens
        for p, v in info.items():
            if v[0] == OPTIONAL and v[1] == o:
                validity[p].append(0)
            if v[0] == REPEATED and v[2] == o:
                offsets[p].append(count[p])

    def present(p):
        rep = info[p][0]
        if rep == REPEATED:
            count[p] += 1
            new_instance(p)
        elif rep == OPTIONAL:
            validity[p][-1] = 1

    for e in ev:
        if e[0] == "startMessage":
            records += 1
            new_instance("")
        elif e[0] == "start":
            present(e[1])
        elif e[0] == "value":
            present(e[1])
    for p in offsets:
        offsets[p].append(count[p])
    return {"records": records, "validity": validity, "offsets": offsets}
