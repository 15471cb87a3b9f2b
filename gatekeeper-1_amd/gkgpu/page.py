"""Bulk form of one audit List page (include/gkgpu.h gk_batch_stage_page).

The audit loop reviews `objList.Items` page by page (pkg/audit/manager.go:341-398)
and looks each object's Namespace up in nsCache (:96-115).  A Page carries the
same data as three flat buffers the engine parses on many host threads:
concatenated object JSON texts with n + 1 byte offsets, the page's distinct
Namespace objects with their offsets, and per object the index of its
Namespace (NO_NS for cluster-scoped objects, reviewed with an empty
corev1.Namespace{}, pkg/target/target.go:137-139).
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

NO_NS = 0xFFFFFFFF


def _text(x) -> str:
    return x if isinstance(x, str) else json.dumps(x, separators=(",", ":"))


def _pack(texts: Sequence[str]):
    """(utf-8 bytes of the concatenation, uint64 offsets[n + 1])"""
    joined = "".join(texts)
    offs = np.zeros(len(texts) + 1, dtype=np.uint64)
    if joined.isascii():
        buf = joined.encode("ascii")
        if texts:
            np.cumsum(np.fromiter(map(len, texts), dtype=np.uint64, count=len(texts)), out=offs[1:])
        return buf, offs
    enc = [t.encode("utf-8", "surrogateescape") for t in texts]
    if enc:
        np.cumsum(np.fromiter(map(len, enc), dtype=np.uint64, count=len(enc)), out=offs[1:])
    return b"".join(enc), offs


@dataclass
class Page:
    objs: bytes
    obj_offs: np.ndarray     # uint64, n + 1
    nss: bytes
    ns_offs: np.ndarray      # uint64, n_ns + 1
    obj_ns: np.ndarray       # uint32, n (NO_NS = cluster-scoped)

    @property
    def n(self) -> int:
        return len(self.obj_offs) - 1

    @property
    def n_ns(self) -> int:
        return len(self.ns_offs) - 1

    @staticmethod
    def from_lists(objs: Sequence, namespaces: Sequence[Optional[object]]) -> "Page":
        """objs: JSON texts or dicts; namespaces: per object its Namespace object
        (JSON text or dict; equal texts / the same object share one entry) or None."""
        if len(objs) != len(namespaces):
            raise ValueError("objs and namespaces differ in length")
        texts = [_text(o) for o in objs]
        table, idx = {}, np.empty(len(objs), dtype=np.uint32)
        ns_texts = []
        for i, ns in enumerate(namespaces):
            if ns is None:
                idx[i] = NO_NS
                continue
            key = ns if isinstance(ns, str) else id(ns)
            k = table.get(key)
            if k is None:
                k = table[key] = len(ns_texts)
                ns_texts.append(_text(ns))
            idx[i] = k
        ob, oo = _pack(texts)
        nb, no = _pack(ns_texts)
        return Page(ob, oo, nb, no, idx)

    def slice(self, lo: int, hi: int) -> "Page":
        """objects [lo, hi) with the whole namespace table"""
        a, b = int(self.obj_offs[lo]), int(self.obj_offs[hi])
        return Page(self.objs[a:b], self.obj_offs[lo:hi + 1] - self.obj_offs[lo], self.nss, self.ns_offs,
                    self.obj_ns[lo:hi].copy())
