"""Nested records for the record-assembly tests: random records of a schema (oracle.assembly.Node
trees), Dremel shredding into per-leaf (r, d, value) stripes as parquet-mr's record writer emits them
(MessageColumnIO's RecordConsumer -> ColumnWriter.write(value, r, d); checked against
TestColumnIO.testWriteWithGroupWriter's expected stripes), and records rebuilt from the automaton's
events. A record is a dict: name -> value (leaf), dict (group), list (REPEATED node), absent (null)."""
import numpy as np

from oracle import assembly as A


def random_record(roots, rng, p_present=0.7, max_rep=3):
    def gen(n):
        if n.repetition == A.REPEATED:
            return [one(n) for _ in range(int(rng.integers(0, max_rep + 1)))]
        if n.repetition == A.OPTIONAL and rng.random() > p_present:
            return None
        return one(n)

    def one(n):
        if not n.children:
            return int(rng.integers(-1000, 1000))
        out = {}
        for c in n.children:
            v = gen(c)
            if v is not None and v != []:
                out[c.name] = v
            elif c.repetition == A.REQUIRED:  # a required field is always there
                out[c.name] = one(c)
        return out
    rec = {}
    for n in roots:
        v = gen(n)
        if v is not None and v != []:
            rec[n.name] = v
        elif n.repetition == A.REQUIRED:
            rec[n.name] = one(n)
    return rec


def shred(roots, records):
    """Per leaf (schema order): (rep_levels, def_levels, dense values)."""
    leaves = A.schema_leaves(roots)
    out = []
    for chain in leaves:
        rl, dl, vals = [], [], []
        lv = A.levels_of([n.repetition for n in chain])

        def visit(obj, k, r, d):
            node = chain[k]
            v = obj.get(node.name) if obj is not None else None
            items = v if node.repetition == A.REPEATED else ([] if v is None else [v])
            if not items:
                rl.append(r)
                dl.append(d)
                return
            for j, it in enumerate(items):
                rr = r if j == 0 else lv[k][0]
                if k == len(chain) - 1:
                    rl.append(rr)
                    dl.append(lv[k][1])
                    vals.append(it)
                else:
                    visit(it, k + 1, rr, lv[k][1])
        for rec in records:
            visit(rec, 0, 0, 0)
        out.append((np.array(rl, dtype=np.uint8), np.array(dl, dtype=np.uint8), vals))
    return out


def rebuild(roots, events):
    """Records from the automaton's converter events (a GroupRecordConverter's view)."""
    reps = {}

    def walk(n, prefix):
        p = prefix + n.name
        reps[p] = n.repetition
        for c in n.children:
            walk(c, p + ".")
    for r in roots:
        walk(r, "")
    records, stack = [], []

    def put(parent, name, val, rep):
        if rep == A.REPEATED:
            parent.setdefault(name, []).append(val)
        else:
            parent[name] = val
    for e in events:
        if e[0] == "startMessage":
            stack = [{}]
        elif e[0] == "endMessage":
            records.append(stack[0])
        elif e[0] == "start":
            g = {}
            put(stack[-1], e[1].rsplit(".", 1)[-1], g, reps[e[1]])
            stack.append(g)
        elif e[0] == "end":
            stack.pop()
        else:
            put(stack[-1], e[1].rsplit(".", 1)[-1], e[2], reps[e[1]])
    return records


def flat_schema(roots):
    """(parent index, repetition) per node in depth-first order, the leaf node indices, and dotted names."""
    nodes, leaf_idx, names = [], [], []

    def walk(n, parent, prefix):
        k = len(nodes)
        nodes.append((parent, n.repetition))
        names.append(prefix + n.name)
        if not n.children:
            leaf_idx.append(k)
        for c in n.children:
            walk(c, k, prefix + n.name + ".")
    for r in roots:
        walk(r, -1, "")
    return nodes, leaf_idx, names
