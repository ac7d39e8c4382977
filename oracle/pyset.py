"""CPython 3.10 set-table emulation for int keys (test infrastructure: the oracle for the order in
which the reference's networkx subgraph views iterate their nodes; csrc/mz_difficulty.hip and
csrc/mz_mcclendon.hip restate the same table in C++ / HIP).

Follows Objects/setobject.c of CPython 3.10 (the interpreter the reference ran on here):
  set_add_entry      probe i = hash & mask, then the LINEAR_PROBES = 9 following slots when
                     i + 9 <= mask, then perturb >>= 5, i = (5 i + 1 + perturb) & mask; insert at
                     the first empty slot; resize when fill * 5 >= mask * 3 to used * 4;
  set_table_resize   the smallest power of two (>= 8) above minused; entries re-inserted in old
                     table order by set_insert_clean (same probe sequence, no equality test); a
                     "resize" to 8 of a set still in its 8-slot small table does nothing;
  set_merge          (set(s), s.union(t), s.update(t) with a set argument): one resize to
                     (used + other.used) * 2 first when (fill + other.used) * 5 >= mask * 3; into
                     an empty set of the same mask as the (dummy-free) source: slot-for-slot copy;
                     into an empty set: set_insert_clean in source table order; otherwise
                     set_add_entry in source table order.
hash(n) == n for the non-negative ints used here (< 2**61 - 1). No deletions occur in the
reference's sets of interest, so there are never dummy entries.
"""

LINEAR_PROBES = 9
PERTURB_SHIFT = 5
MINSIZE = 8


class PySet:
    __slots__ = ("table", "mask", "fill", "used", "small")

    def __init__(self):
        self.table = [None] * MINSIZE
        self.mask = MINSIZE - 1
        self.fill = self.used = 0
        self.small = True  # still in the 8-slot smalltable

    # ---- setobject.c primitives ---------------------------------------------------------------
    @staticmethod
    def _insert_clean(table, mask, key):
        perturb = key
        i = key & mask
        while True:
            if table[i] is None:
                table[i] = key
                return
            if i + LINEAR_PROBES <= mask:
                for j in range(1, LINEAR_PROBES + 1):
                    if table[i + j] is None:
                        table[i + j] = key
                        return
            perturb >>= PERTURB_SHIFT
            i = (i * 5 + 1 + perturb) & mask

    def _resize(self, minused):
        newsize = MINSIZE
        while newsize <= minused:
            newsize <<= 1
        if newsize == MINSIZE and self.small:
            return  # no dummies: nothing to do
        old = self.table
        self.table = [None] * newsize
        self.mask = newsize - 1
        self.small = newsize == MINSIZE
        for k in old:
            if k is not None:
                self._insert_clean(self.table, self.mask, k)
        self.fill = self.used

    def add(self, key):
        mask = self.mask
        i = key & mask
        perturb = key
        while True:
            probes = LINEAR_PROBES if i + LINEAR_PROBES <= mask else 0
            e = i
            while True:
                k = self.table[e]
                if k is None:
                    self.table[e] = key
                    self.fill += 1
                    self.used += 1
                    if self.fill * 5 >= mask * 3:
                        self._resize(self.used * 4 if self.used <= 50000 else self.used * 2)
                    return
                if k == key:
                    return
                if probes == 0:
                    break
                probes -= 1
                e += 1
            perturb >>= PERTURB_SHIFT
            i = (i * 5 + 1 + perturb) & mask

    def merge(self, other):
        """set_merge(self, other) for a set `other`."""
        if other is self or other.used == 0:
            return
        if (self.fill + other.used) * 5 >= self.mask * 3:
            self._resize((self.used + other.used) * 2)
        if self.fill == 0 and self.mask == other.mask:
            self.table = list(other.table)
            self.fill, self.used = other.fill, other.used
            return
        if self.fill == 0:
            for k in other.table:
                if k is not None:
                    self._insert_clean(self.table, self.mask, k)
            self.fill = self.used = other.used
            return
        for k in other.table:
            if k is not None:
                self.add(k)

    # ---- Python-level operations --------------------------------------------------------------
    @classmethod
    def from_iter(cls, keys):
        """set(iterable) of a non-set iterable / a set display + add() calls."""
        s = cls()
        for k in keys:
            s.add(k)
        return s

    def copy(self):
        """set(s) / s.copy() / the first step of s.union(...)."""
        s = PySet()
        s.merge(self)
        return s

    def union(self, other):
        s = self.copy()
        s.merge(other)
        return s

    def __iter__(self):
        return (k for k in self.table if k is not None)

    def __len__(self):
        return self.used

    def __contains__(self, key):
        return key in set(self)
