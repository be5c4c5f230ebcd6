#!/usr/bin/env python3
"""Generate tests/golden/ref_net.json from the reference's own dns.c,
address.c, packet.c and payload.c, compiled unmodified into
oracle/_ref/libshdref_net.so (oracle/Makefile `ref`; harness
oracle/ref_harness/ref_net.c).  Run in the build container, where
/root/reference exists:  make -C oracle ref && python3 tests/golden/make_ref_net.py

The fixture holds
* dns: per case, the iphint of each host in registration order (null: no
  hint) and the ethernet address dns_register gave it (host.c:166-167,
  dns.c:102-134), as a dotted string;
* status: per scripted UDP packet object (host id, packet id, addresses,
  ports, payload, the status calls in order, then its release) the lines
  packet_addDeliveryStatus logs (packet.c:647-659), one per call, the last
  one PDS_DESTROYED (packet_unref, packet.c:194-201).
"""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "shadow-1_amd"))
LIB = os.path.join(REPO, "oracle", "_ref", "libshdref_net.so")

import shdgpu as S  # noqa: E402  (STATUS_FLAG: packet.h's values)

# the config front-end test's hosts (tests/test_config_cpu.py CONFIG), then
# hints that exercise each rule of dns_register / _dns_isRestricted
DNS_CASES = [
    ["11.0.0.3", "11.0.0.3", "11.0.0.3", None, "10.1.2.3", "127.0.0.1", "not-an-ip", "52.0.0.7", "52.0.0.7"],
    ["11.0.0.1", None, "11.0.0.2", "100.64.0.1", "100.63.255.255", "255.255.255.255", "0.0.0.0", "11.0.0.5",
     "1.2.3.4", None, "011.0.0.1", "11.0.1.0", "192.168.1.1", "172.31.0.1", "172.32.0.1", "224.0.0.1",
     "223.255.255.255", "198.18.0.5", "198.20.0.5", "169.254.3.3", "11.0.0.12", None, None, " 11.0.0.40",
     "11.0.0.40", "11.0.0.255", "11.0.1.1"],
    [None] * 300 + ["11.0.1.45", "11.0.0.200", None],
]


SEND = ["SND_CREATED", "SND_SOCKET_BUFFERED", "SND_INTERFACE_SENT"]
RECV = ["ROUTER_DEQUEUED", "RCV_INTERFACE_RECEIVED", "RCV_SOCKET_PROCESSED", "RCV_SOCKET_BUFFERED"]
# One packet OBJECT's life each (the harness releases it at the end: its
# PDS_DESTROYED line closes the story).  From INET_SENT on a sent datagram is
# two objects (worker.c:306-313): "orig" (released by the sender at once,
# network_interface.c:577) and "copy" (the receiver's).
A = dict(host_id=7, pkt=5, src="11.0.0.1", sport=12345, dst="11.0.0.2", dport=8998, payload=1)
B = dict(host_id=3, pkt=0, src="11.0.0.9", sport=10000, dst="11.0.3.7", dport=8998, payload=1)
C_ = dict(host_id=4294967295, pkt=4294967294, src="52.0.0.7", sport=65535, dst="11.0.0.1", dport=8998,
          payload=1500)
D = dict(host_id=12, pkt=99, src="11.0.0.2", sport=40000, dst="11.0.0.3", dport=8998, payload=1500)
E = dict(host_id=8, pkt=0, src="11.0.0.2", sport=10001, dst="11.0.0.2", dport=8998, payload=1)
F = dict(host_id=1, pkt=1, src="100.0.0.1", sport=1, dst="11.0.0.1", dport=8998, payload=0)
STORIES = [
    dict(A, role="orig", statuses=SEND + ["INET_SENT"]),
    dict(A, role="copy", statuses=SEND + ["INET_SENT", "ROUTER_ENQUEUED"] + RECV + ["RCV_SOCKET_DELIVERED"]),
    dict(B, role="orig", statuses=SEND + ["INET_DROPPED"]),                       # dropped on the path
    dict(C_, role="orig", statuses=SEND + ["INET_SENT"]),
    dict(C_, role="copy", statuses=SEND + ["INET_SENT", "ROUTER_ENQUEUED", "ROUTER_DROPPED"]),   # CoDel
    dict(D, role="orig", statuses=SEND + ["INET_SENT"]),
    dict(D, role="copy", statuses=SEND + ["INET_SENT", "ROUTER_ENQUEUED", "ROUTER_DEQUEUED",      # no listener
                                          "RCV_INTERFACE_RECEIVED", "RCV_INTERFACE_DROPPED"]),
    dict(E, role="loop", statuses=SEND + RECV[1:] + ["RCV_SOCKET_DELIVERED"]),   # loopback: one object
    dict(F, role="orig", statuses=SEND + ["INET_SENT"]),                         # an empty datagram
    dict(F, role="copy", statuses=SEND + ["INET_SENT"]),                         # its copy dropped at push
    # the widest packet id (guint64, packet.c:522)
    dict(A, pkt=18446744073709551615, role="format", statuses=SEND + ["INET_DROPPED"]),
]


def ip_u32(s):
    a = [int(x) for x in s.split(".")]
    return (a[0] << 24) | (a[1] << 16) | (a[2] << 8) | a[3]


def lib():
    l = C.CDLL(LIB)
    l.ref_dns_assign.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_uint32)]
    l.ref_status_story.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.POINTER(C.c_uint32), C.c_int, C.c_char_p, C.c_size_t]
    return l


def ref_dns(l, hints):
    n = len(hints)
    arr = (C.c_char_p * n)(*[None if h is None else h.encode() for h in hints])
    out = (C.c_uint32 * n)()
    assert l.ref_dns_assign(n, arr, out) == 0
    return [S.ip_string(int(x)) for x in out]


def ref_story(l, st):
    flags = (C.c_uint32 * len(st["statuses"]))(*[S.STATUS_FLAG[x] for x in st["statuses"]])
    # (the harness's packet_unref at the end adds the PDS_DESTROYED line)
    buf = C.create_string_buffer(1 << 16)
    rc = l.ref_status_story(st["host_id"], st["pkt"], ip_u32(st["src"]), st["sport"], ip_u32(st["dst"]),
                            st["dport"], st["payload"], flags, len(st["statuses"]), buf, len(buf))
    assert rc == 0
    return buf.value.decode().rstrip("\n").split("\n")


def main():
    l = lib()
    fx = {
        "generator": "tests/golden/make_ref_net.py over oracle/_ref/libshdref_net.so "
                     "(reference dns.c, address.c, packet.c, payload.c compiled unmodified)",
        "dns": [dict(hints=h, ips=ref_dns(l, h)) for h in DNS_CASES],
        "status": [dict(story=s, lines=ref_story(l, s)) for s in STORIES],
    }
    with open(os.path.join(HERE, "ref_net.json"), "w") as f:
        json.dump(fx, f, indent=1)
    print("wrote ref_net.json:", len(fx["dns"]), "dns cases,", len(fx["status"]), "stories")


if __name__ == "__main__":
    main()
