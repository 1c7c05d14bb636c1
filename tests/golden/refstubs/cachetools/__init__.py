"""Stand-in for ``cachetools`` (unpinned, run_savio.sh:39): an LRU with the
eviction semantics the reference's CacheDict relies on (src/cache_dict.py:42).
Fixture-generation infrastructure only.  ``GM_LRU_UNBOUNDED=1`` disables
eviction (used to show the reference's lost-append defect is LRU-induced)."""
import collections
import os


class LRUCache:
    def __init__(self, maxsize):
        self._d = collections.OrderedDict()
        self._max = None if os.environ.get("GM_LRU_UNBOUNDED") == "1" else maxsize

    def __getitem__(self, k):
        v = self._d[k]
        self._d.move_to_end(k)
        return v

    def __setitem__(self, k, v):
        self._d[k] = v
        self._d.move_to_end(k)
        if self._max is not None:
            while len(self._d) > self._max:
                self._d.popitem(last=False)

    def __delitem__(self, k):
        del self._d[k]

    def __contains__(self, k):
        return k in self._d

    def __len__(self):
        return len(self._d)
