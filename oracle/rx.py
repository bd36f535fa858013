"""CPU restatement of the receive-side checks after open — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module, as
the checker for wg_rx_check (wireguard-java_amd/csrc/wg_rx.hip); the product never calls it.

* ``IPFilter`` follows util/IPFilter.java line by line: ``insert`` (:30-42) builds a binary
  trie one bit per level; ``search`` (:49-61) walks the address bits, reporting a match if a
  node it passes *before* descending (depths 0 .. nbits-1) ends a subnet, and stops at the
  first missing child. So /32 and /128 entries never match, and ``allowing_all()``
  (:67-77: 0.0.0.0/32 and ::/128) matches nothing. Pinned by the reference's own expected
  outputs in IPFilter.main (:79-93), tests/golden/rx_vectors.json.
* ``destination_ip`` follows TransportManager.destinationIPOf (:124-130): the version
  nibble of byte 0 (read as a signed Java byte, so 0x80..0xFF give negative values and hit
  the default branch) selects bytes 16..19 (4) or 24..39 (6); anything else throws, and so
  does a slice past the end of the packet.
* ``process_decrypted`` follows TransportManager.processDecryptedTransport (:98-119):
  zero-length = keepalive (not forwarded), else the destination filter decides.
* ``ReplayWindow`` restates the batch window of include/wgaead.h (WG_RX_REPLAY), which the
  reference does not have: parity for it is against this
  restatement only ("parity unpinned" with respect to the reference).
"""
from __future__ import annotations

import ipaddress

PKT_OK, PKT_BADTAG, PKT_KEEPALIVE, PKT_BADIP, PKT_FILTERED, PKT_REPLAY = 0, 1, 3, 4, 5, 6
REJECT_AFTER = (1 << 64) - (1 << 13) - 1


class _Node:
    __slots__ = ("children", "end")

    def __init__(self):
        self.children = [None, None]
        self.end = False


def _bit(b: bytes, i: int) -> int:
    return (b[i // 8] >> (7 - i % 8)) & 1


class IPFilter:
    """util/IPFilter.java restated."""

    def __init__(self):
        self.root4 = _Node()
        self.root6 = _Node()

    def insert(self, addr, prefix_len: int) -> None:  # :30-42
        b = ipaddress.ip_address(addr).packed if isinstance(addr, str) else bytes(addr)
        node = self.root4 if len(b) == 4 else self.root6
        for i in range(prefix_len):
            bit = _bit(b, i)
            if node.children[bit] is None:
                node.children[bit] = _Node()
            node = node.children[bit]
        node.end = True

    def search(self, ip: bytes) -> bool:  # :49-61
        node = self.root4 if len(ip) == 4 else self.root6
        found = False
        for i in range(len(ip) * 8):
            if node.end:
                found = True
            node = node.children[_bit(ip, i)]
            if node is None:
                break
        return found

    @staticmethod
    def allowing_all() -> "IPFilter":  # :67-77
        f = IPFilter()
        f.insert("0.0.0.0", 32)
        f.insert("::", 128)
        return f


def destination_ip(pt: bytes):
    """TransportManager.destinationIPOf (:124-130); None where the reference throws."""
    v = pt[0] if pt[0] < 128 else pt[0] - 256  # JAVA_BYTE is signed
    v >>= 4
    if v == 4:
        return pt[16:20] if len(pt) >= 20 else None
    if v == 6:
        return pt[24:40] if len(pt) >= 40 else None
    return None


def process_decrypted(pt: bytes, flt: IPFilter | None) -> int:
    """processDecryptedTransport (:98-119) as a status: OK = forwarded to the tun queue."""
    if len(pt) == 0:
        return PKT_KEEPALIVE
    dst = destination_ip(pt)
    if dst is None:
        return PKT_BADIP
    if flt is not None and not flt.search(dst):
        return PKT_FILTERED
    return PKT_OK


class ReplayWindow:
    """Per key slot: top = highest accepted counter + 1, set of accepted counters within
    [top - W, top). ``check_batch`` applies one batch against the window as it stood
    before the batch, then advances it (include/wgaead.h, WG_RX_REPLAY)."""

    def __init__(self, window_bits: int):
        self.W = window_bits
        self.top = {}
        self.seen = {}

    def reset(self, slot: int) -> None:
        self.top.pop(slot, None)
        self.seen.pop(slot, None)

    def check_batch(self, slots, counters, status) -> list[int]:
        st = list(status)
        first = {}
        for i, s in enumerate(slots):
            if st[i] == PKT_OK:
                first.setdefault((int(s), int(counters[i])), i)
        accepted = []
        for i, s in enumerate(slots):
            if st[i] != PKT_OK:
                continue
            s, c = int(s), int(counters[i])
            top = self.top.get(s, 0)
            ok = c < REJECT_AFTER and first[(s, c)] == i
            if ok and c < top:
                ok = top - c <= self.W and c not in self.seen.get(s, set())
            if ok:
                accepted.append((s, c))
            else:
                st[i] = PKT_REPLAY
        for s, c in accepted:
            self.top[s] = max(self.top.get(s, 0), c + 1)
        for s, c in accepted:
            self.seen.setdefault(s, set()).add(c)
        for s in {s for s, _ in accepted}:
            t = self.top[s]
            self.seen[s] = {c for c in self.seen[s] if t - c <= self.W}
        return st

    def bitmap(self, slot: int):
        """(top, words) in the device layout: bit (c mod W) of word (c mod W) // 64."""
        words = [0] * (self.W // 64)
        for c in self.seen.get(slot, set()):
            p = c % self.W
            words[p // 64] |= 1 << (p % 64)
        return self.top.get(slot, 0), words


def rx_check(slots, counters, lengths, plaintexts, status, filters_of_slot, window: ReplayWindow | None,
             do_filter: bool = True) -> list[int]:
    """wg_rx_check restated: replay window (if given) on the authenticated packets, then the
    keepalive / destination checks on the survivors. filters_of_slot: slot -> IPFilter or
    None (no filter: every destination passes)."""
    st = list(status)
    if window is not None:
        st = window.check_batch(slots, counters, st)
    if do_filter:
        for i in range(len(st)):
            if st[i] == PKT_OK:
                st[i] = process_decrypted(plaintexts[i][:int(lengths[i])], filters_of_slot.get(int(slots[i])))
    return st
