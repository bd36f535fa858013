"""Receive-side restatement (oracle/rx.py) against the reference's own known answers
(IPFilter.main, util/IPFilter.java:79-93) and the behaviour its code implies; the replay
window's batch rules (include/wgaead.h, WG_RX_REPLAY) on hand-made sequences."""
import ipaddress
import json
import os

from oracle import rx
from wgtest import ROOT

G = json.load(open(os.path.join(ROOT, "tests", "golden", "rx_vectors.json")))


def _ip(s):
    return ipaddress.ip_address(s).packed


def test_ipfilter_reference_known_answers():
    f = rx.IPFilter()
    for a, p in G["filter"]:
        f.insert(a, p)
    for a, want in G["search"]:
        assert f.search(_ip(a)) is want, a


def test_ipfilter_full_length_prefixes_never_match():
    """search() tests a node before descending, so the depth-32 / depth-128 node of a /32 or
    /128 entry is never tested: allowingAll() (0.0.0.0/32, ::/128) lets nothing through."""
    f = rx.IPFilter.allowing_all()
    for a in ("0.0.0.0", "1.2.3.4", "::", "2001:db8::1"):
        assert not f.search(_ip(a))
    g = rx.IPFilter()
    g.insert("10.0.0.1", 32)
    assert not g.search(_ip("10.0.0.1"))
    g.insert("10.0.0.0", 31)
    assert g.search(_ip("10.0.0.1")) and g.search(_ip("10.0.0.0")) and not g.search(_ip("10.0.0.2"))
    z = rx.IPFilter()
    z.insert("0.0.0.0", 0)  # /0: the root ends a subnet -> every IPv4 address
    assert z.search(_ip("255.1.2.3")) and not z.search(_ip("::1"))


def test_destination_and_process_decrypted():
    v4 = bytes([0x45]) + bytes(15) + _ip("192.168.1.9") + bytes(8)
    v6 = bytes([0x60]) + bytes(23) + _ip("2001:db8::5") + bytes(4)
    assert rx.destination_ip(v4) == _ip("192.168.1.9")
    assert rx.destination_ip(v6) == _ip("2001:db8::5")
    assert rx.destination_ip(bytes([0x45]) + bytes(18)) is None       # 19 bytes: slice throws
    assert rx.destination_ip(bytes([0x85]) + bytes(40)) is None       # signed byte: -8
    assert rx.destination_ip(bytes([0x50]) + bytes(40)) is None
    f = rx.IPFilter()
    for a, p in G["filter"]:
        f.insert(a, p)
    assert rx.process_decrypted(b"", f) == rx.PKT_KEEPALIVE
    assert rx.process_decrypted(v4, f) == rx.PKT_OK
    assert rx.process_decrypted(v6, f) == rx.PKT_OK
    assert rx.process_decrypted(v4.replace(_ip("192.168.1.9"), _ip("192.168.2.9")), f) == rx.PKT_FILTERED
    assert rx.process_decrypted(v4, None) == rx.PKT_OK


def test_replay_window_rules():
    w = rx.ReplayWindow(128)
    ok, rp = rx.PKT_OK, rx.PKT_REPLAY
    # batch 1: in order, one duplicate (second copy rejected), a bad tag stays bad
    st = w.check_batch([0] * 5, [0, 1, 2, 1, 3], [ok, ok, ok, ok, rx.PKT_BADTAG])
    assert st == [ok, ok, ok, rp, rx.PKT_BADTAG]
    assert w.top[0] == 3
    # batch 2: replay of 0, a gap fill-in later, the far future, Reject-After
    st = w.check_batch([0] * 4, [0, 500, 3, rx.REJECT_AFTER], [ok] * 4)
    assert st == [rp, ok, ok, rp]
    assert w.top[0] == 501
    # batch 3: 3 is now older than the window (501 - 3 > 128); 400 is inside and unseen
    st = w.check_batch([0, 0, 0], [3, 400, 500], [ok] * 3)
    assert st == [rp, ok, rp]
    # other slots are independent; reset empties a slot
    assert w.check_batch([1], [0], [ok]) == [ok]
    w.reset(0)
    assert w.check_batch([0], [0], [ok]) == [ok]


def test_replay_window_slides_between_batches():
    """Within one batch the window is the one before the batch: 10 is accepted after 1000 in
    the same batch (W = 64), and rejected in the next batch."""
    w = rx.ReplayWindow(64)
    ok = rx.PKT_OK
    assert w.check_batch([0, 0, 0], [20, 1000, 10], [ok] * 3) == [ok, ok, ok]
    assert w.check_batch([0], [11], [ok]) == [rx.PKT_REPLAY]
    top, words = w.bitmap(0)
    assert top == 1001 and sum(bin(x).count("1") for x in words) == 1  # only 1000 is inside
