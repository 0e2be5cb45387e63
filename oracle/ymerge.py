"""oracle/ymerge.py — CPU restatement of Y.mergeUpdates / Y.diffUpdate (Yjs 13.5.16, update v1).

TEST INFRASTRUCTURE ONLY: imported by tests/ (and never by the product path). It restates, step
for step, the lazy k-way merge of the in-image Yjs bundle:

    lazyStructReaderGenerator  Y@36564   structs of one update; items keep parentSub only when
                                         they carry neither origin nor right origin
    LazyStructReader           Y@37152   (filterSkips drops Skip structs of merge inputs)
    sliceStruct                Y@38665   `as`: GC / Skip / Item cut at an offset
    mergeUpdatesV2             Y@39011   `ds`: readers re-sorted every step (client desc, clock asc,
                                         non-Skip first) with a STABLE sort, as V8's Array.sort
    diffUpdateV2               Y@40711   `us`
    LazyStructWriter           Y@41394.. `rs` / `ps` / `gs` / `ws`
    mergeDeleteSets            Y@10486   `he` (+ sortAndMergeDeleteSet `le`, writeDeleteSet `fe`)

Content is kept as raw element byte strings (Any / JSON) or raw bytes, so writes are byte copies;
this equals Yjs's re-encoding for Yjs-produced (canonical lib0) input. Pinned against the
`merged_raw` fields of tests/golden/*.json (Yjs's own mergeUpdates output).
"""

# ---------------------------------------------------------------------------- lib0 primitives
class Dec:
    def __init__(self, b):
        self.b = b
        self.p = 0

    def u8(self):
        if self.p >= len(self.b):
            raise ValueError("Integer out of range!")
        v = self.b[self.p]
        self.p += 1
        return v

    def vu(self):  # readVarUint, lib0 0.2.42 (32-bit accumulation)
        v = 0
        shift = 0
        while True:
            r = self.u8()
            if shift < 32:
                v |= (r & 0x7F) << shift
            v &= 0xFFFFFFFF
            shift += 7
            if r < 0x80:
                return v
            if shift > 35:
                raise ValueError("Integer out of range!")

    def raw(self, n):
        if self.p + n > len(self.b):
            raise ValueError("Integer out of range!")
        s = self.b[self.p:self.p + n]
        self.p += n
        return s

    def vstr_raw(self):  # varString incl. its length prefix
        st = self.p
        n = self.vu()
        self.raw(n)
        return self.b[st:self.p]

    def vi(self):
        r = self.u8()
        if r & 0x80:
            while True:
                r = self.u8()
                if r < 0x80:
                    break

    def any_raw(self):
        st = self.p
        self._any()
        return self.b[st:self.p]

    def _any(self):
        # readAny (L0@1937) recurses without a limit: an explicit stack of [members left, is object]
        stack = []
        while True:
            t = self.u8()
            if t in (127, 126, 121, 120):
                pass
            elif t == 125:
                self.vi()
            elif t == 124:
                self.raw(4)
            elif t in (123, 122):
                self.raw(8)
            elif t in (119, 116):
                self.raw(self.vu())
            elif t in (117, 118):
                n = self.vu()
                if n:
                    stack.append([n, t == 118])
                    if t == 118:
                        self.vstr_raw()
                    continue
            else:
                raise ValueError("Unexpected case")
            while stack:  # a value completed: the next member of the innermost open container
                top = stack[-1]
                top[0] -= 1
                if top[0]:
                    if top[1]:
                        self.vstr_raw()
                    break
                stack.pop()
            if not stack:
                return


def wvu(out, v):
    while v > 0x7F:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)


def utf16_len(b):
    s = b.decode("utf-8")
    return sum(2 if ord(c) > 0xFFFF else 1 for c in s)


def utf16_slice(b, off):
    s = b.decode("utf-8")
    units = 0
    for i, c in enumerate(s):
        if units == off:
            return s[i:].encode("utf-8")
        units += 2 if ord(c) > 0xFFFF else 1
        if units > off:
            raise ValueError("slice inside a surrogate pair (lone surrogate: lib0 0.2.42 throws)")
    return b""


# ---------------------------------------------------------------------------- structs
GC, SKIP, ITEM = 0, 10, 1


class Struct:
    __slots__ = ("kind", "client", "clock", "length", "ref", "origin", "right_origin", "parent", "parent_sub", "content")

    def __init__(self, kind, client, clock, length, ref=0, origin=None, right_origin=None, parent=None, parent_sub=None,
                 content=None):
        self.kind, self.client, self.clock, self.length = kind, client, clock, length
        self.ref, self.origin, self.right_origin = ref, origin, right_origin
        self.parent, self.parent_sub, self.content = parent, parent_sub, content

    def end(self):
        return self.clock + self.length

    # Item.write / GC.write / Skip.write with writeStructs offset (Y@80416, Y@68955)
    def write(self, out, offset):
        if self.kind != ITEM:
            out.append(self.kind)
            wvu(out, self.length - offset)
            return
        origin = (self.client, self.clock + offset - 1) if offset > 0 else self.origin
        info = self.ref | (0x80 if origin is not None else 0) | (0x40 if self.right_origin is not None else 0) | \
            (0x20 if self.parent_sub is not None else 0)
        out.append(info)
        if origin is not None:
            wvu(out, origin[0])
            wvu(out, origin[1])
        if self.right_origin is not None:
            wvu(out, self.right_origin[0])
            wvu(out, self.right_origin[1])
        if origin is None and self.right_origin is None:
            if isinstance(self.parent, bytes):
                out.append(1)
                out += self.parent
            else:
                out.append(0)
                wvu(out, self.parent[0])
                wvu(out, self.parent[1])
            if self.parent_sub is not None:
                out += self.parent_sub
        c = self.content
        if self.ref == 1:
            wvu(out, self.length - offset)
        elif self.ref in (2, 8):
            wvu(out, self.length - offset)
            for e in c[offset:]:
                out += e
        elif self.ref == 4:
            s = utf16_slice(c, offset)
            wvu(out, len(s))
            out += s
        else:
            out += c


def read_content(d, info):
    ref = info & 31
    if ref == 1:
        n = d.vu()
        return n, None
    if ref == 2:
        n = d.vu()
        return n, [d.vstr_raw() for _ in range(n)]
    if ref == 3:
        return 1, d.vstr_raw()
    if ref == 4:
        s = d.raw(d.vu())
        return utf16_len(s), s
    if ref in (5,):
        return 1, d.vstr_raw()
    if ref == 6:
        st = d.p
        d.vstr_raw()
        d.vstr_raw()
        return 1, d.b[st:d.p]
    if ref == 7:
        st = d.p
        tr = d.vu()
        if tr in (3, 5):
            d.vstr_raw()
        return 1, d.b[st:d.p]
    if ref == 8:
        n = d.vu()
        return n, [d.any_raw() for _ in range(n)]
    if ref == 9:
        st = d.p
        d.vstr_raw()
        d.any_raw()
        return 1, d.b[st:d.p]
    raise ValueError("Unexpected case")


def lazy_structs(d):
    """lazyStructReaderGenerator (Y@36564)."""
    out = []
    for _ in range(d.vu()):
        n = d.vu()
        client = d.vu()
        clock = d.vu()
        for _ in range(n):
            info = d.u8()
            ref = info & 31
            if ref == SKIP:
                ln = d.vu()
                out.append(Struct(SKIP, client, clock, ln))
                clock += ln
            elif ref != 0:
                origin = (d.vu(), d.vu()) if info & 0x80 else None
                right = (d.vu(), d.vu()) if info & 0x40 else None
                cant_copy = (info & 0xC0) == 0
                parent = psub = None
                if cant_copy:
                    if d.vu() == 1:
                        parent = d.vstr_raw()
                    else:
                        parent = (d.vu(), d.vu())
                    if info & 0x20:
                        psub = d.vstr_raw()
                ln, content = read_content(d, info)
                out.append(Struct(ITEM, client, clock, ln, ref, origin, right, parent, psub, content))
                clock += ln
            else:
                ln = d.vu()
                out.append(Struct(GC, client, clock, ln))
                clock += ln
    return out


def read_delete_set(d):
    """readDeleteSet (Y@11105 `ge`): Map<client, [(clock, len)]> in wire order."""
    ds = {}
    for _ in range(d.vu()):
        client = d.vu()
        n = d.vu()
        if n > 0:
            lst = ds.setdefault(client, [])
            for _ in range(n):
                lst.append([d.vu(), d.vu()])
    return ds


def merge_delete_sets(dss):
    """mergeDeleteSets (`he`) + sortAndMergeDeleteSet (`le`)."""
    res = {}
    for i, ds in enumerate(dss):
        for client, ranges in ds.items():
            if client not in res:
                lst = [list(r) for r in ranges]
                for ds2 in dss[i + 1:]:
                    lst += [list(r) for r in ds2.get(client, [])]
                res[client] = lst
    for client, lst in res.items():
        lst.sort(key=lambda r: r[0])
        n = 1
        for e in range(1, len(lst)):
            s, r = lst[n - 1], lst[e]
            if s[0] + s[1] >= r[0]:
                s[1] = max(s[1], r[0] + r[1] - s[0])
            else:
                lst[n] = r
                n += 1
        del lst[n:]
    return res


def write_delete_set(out, ds):
    wvu(out, len(ds))
    for client, ranges in ds.items():
        wvu(out, client)
        wvu(out, len(ranges))
        for c, ln in ranges:
            wvu(out, c)
            wvu(out, ln)


def slice_struct(s, e):
    """sliceStruct (Y@38665 `as`)."""
    if s.kind != ITEM:
        return Struct(s.kind, s.client, s.clock + e, s.length - e)
    c = s.content
    if s.ref == 1:
        nc = None
    elif s.ref in (2, 8):
        nc = c[e:]
    elif s.ref == 4:
        nc = utf16_slice(c, e)
    else:
        raise ValueError("splice of a length-1 content")
    return Struct(ITEM, s.client, s.clock + e, s.length - e, s.ref, (s.client, s.clock + e - 1), s.right_origin,
                  s.parent, s.parent_sub, nc)


def merge_with(a, b):
    """GC / Skip merge unconditionally; lazily read Items never merge (this.right !== right)."""
    if a.kind != b.kind or a.kind == ITEM:
        return False
    a.length += b.length
    return True


class Writer:
    """LazyStructWriter (`rs`) + writeStructToLazyStructWriter (`ps`) / flush (`gs`) / finish (`ws`)."""

    def __init__(self):
        self.curr_client = 0
        self.written = 0
        self.rest = bytearray()
        self.client_structs = []

    def flush(self):
        if self.written > 0:
            self.client_structs.append((self.written, bytes(self.rest)))
            self.rest = bytearray()
            self.written = 0

    def put(self, s, offset):
        if self.written > 0 and self.curr_client != s.client:
            self.flush()
        if self.written == 0:
            self.curr_client = s.client
            wvu(self.rest, s.client)
            wvu(self.rest, s.clock + offset)
        s.write(self.rest, offset)
        self.written += 1

    def finish(self, out):
        self.flush()
        wvu(out, len(self.client_structs))
        for n, r in self.client_structs:
            wvu(out, n)
            out += r


class Reader:
    def __init__(self, structs, filter_skips):
        self.structs = structs
        self.i = -1
        self.filter_skips = filter_skips
        self.curr = None
        self.next()

    def next(self):
        while True:
            self.i += 1
            self.curr = self.structs[self.i] if self.i < len(self.structs) else None
            if not (self.filter_skips and self.curr is not None and self.curr.kind == SKIP):
                return self.curr


def _cmp_key(r):
    c = r.curr
    return (-c.client, c.clock, 1 if c.kind == SKIP else 0)


def merge_updates(updates):
    """Y.mergeUpdates (mergeUpdatesV2 `ds`, Y@39011) for v1 updates."""
    if len(updates) == 1:
        return bytes(updates[0])
    decs = [Dec(bytes(u)) for u in updates]
    readers = [Reader(lazy_structs(d), True) for d in decs]
    cur = None  # [struct, offset]
    w = Writer()
    while True:
        readers = [r for r in readers if r.curr is not None]
        readers.sort(key=_cmp_key)  # Python's sort is stable, as V8's TimSort
        if not readers:
            break
        t = readers[0]
        e = t.curr.client
        if cur is not None:
            n = t.curr
            skipped = False
            cs = cur[0]
            while n is not None and n.clock + n.length <= cs.clock + cs.length and n.client >= cs.client:
                n = t.next()
                skipped = True
            if n is None or n.client != e or (skipped and n.clock > cs.clock + cs.length):
                continue
            if e != cs.client:
                w.put(cs, cur[1])
                cur = [n, 0]
                t.next()
            else:
                if cs.clock + cs.length < n.clock:
                    if cs.kind == SKIP:
                        cs.length = n.clock + n.length - cs.clock
                    else:
                        w.put(cs, cur[1])
                        gap = n.clock - cs.clock - cs.length
                        cur = [Struct(SKIP, e, cs.clock + cs.length, gap), 0]
                else:
                    diff = cs.clock + cs.length - n.clock
                    if diff > 0:
                        if cs.kind == SKIP:
                            cs.length -= diff
                        else:
                            n = slice_struct(n, diff)
                    if not merge_with(cs, n):
                        w.put(cs, cur[1])
                        cur = [n, 0]
                        t.next()
        else:
            cur = [t.curr, 0]
            t.next()
        n = t.curr
        while n is not None and n.client == e and n.clock == cur[0].clock + cur[0].length and n.kind != SKIP:
            w.put(cur[0], cur[1])
            cur = [n, 0]
            n = t.next()
    if cur is not None:
        w.put(cur[0], cur[1])
    out = bytearray()
    w.finish(out)
    write_delete_set(out, merge_delete_sets([read_delete_set(d) for d in decs]))
    return bytes(out)


def decode_sv(sv):
    d = Dec(bytes(sv))
    m = {}
    for _ in range(d.vu()):
        c = d.vu()
        m[c] = d.vu()
    return m


def diff_update(update, sv):
    """Y.diffUpdate (diffUpdateV2 `us`, Y@40711) for a v1 update and a v1 state vector."""
    state = decode_sv(sv)
    d = Dec(bytes(update))
    r = Reader(lazy_structs(d), False)
    w = Writer()
    while r.curr is not None:
        c = r.curr
        client = c.client
        svc = state.get(client, 0)
        if c.kind == SKIP:
            r.next()
            continue
        if c.clock + c.length > svc:
            w.put(c, max(svc - c.clock, 0))
            r.next()
            while r.curr is not None and r.curr.client == client:
                w.put(r.curr, 0)
                r.next()
        else:
            while r.curr is not None and r.curr.client == client and r.curr.clock + r.curr.length <= svc:
                r.next()
    out = bytearray()
    w.finish(out)
    write_delete_set(out, read_delete_set(d))
    return bytes(out)
