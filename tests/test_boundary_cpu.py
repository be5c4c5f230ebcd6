"""The reference-shaped boundary on the CPU (no compute calls).

* libshdshadow.so (shadow-1_amd/host/topology_shd.c) implements exactly the
  functions of the reference's src/main/routing/topology.h:17-28 and leaves
  Shadow's own address / random / worker functions for Shadow to provide.
* In the build container, where the reference tree is readable, the adapter is
  compiled with the reference header force-included: a signature that drifted
  from topology.h (glib types included) is a compile error.  The same is done
  for the SchedulerPolicy adapter against scheduler_policy.h, whose struct
  layout is compared field by field.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "shadow-1_amd")
TOPO_LIB = os.path.join(PKG, "libshdshadow.so")
REF = "/root/reference/src"
GLIB = ["-I/opt/conda/include/glib-2.0", "-I/opt/conda/lib/glib-2.0/include"]

# topology.h:17-28 (the reference's declarations, by name)
TOPOLOGY_API = {"topology_new", "topology_free", "topology_attach", "topology_detach", "topology_isRoutable",
                "topology_getLatency", "topology_getReliability", "topology_incrementPathPacketCounter"}
SHADOW_PROVIDES = {"address_toHostIP", "random_nextDouble", "worker_updateMinTimeJump", "event_compare",
                   "event_getTime", "event_unref", "g_queue_new", "g_queue_push_tail", "g_queue_free"}


def nm(path, flag):
    out = subprocess.run(["nm", "-D", flag, path], capture_output=True, text=True, check=True).stdout
    return {l.split()[-1].split("@")[0] for l in out.splitlines() if l.strip()}


def have_reference():
    return os.path.isdir(REF) and os.path.isdir(GLIB[0][2:])


def test_topology_adapter_exports_the_reference_api():
    assert os.path.exists(TOPO_LIB), "run __graft_entry__.build()"
    defined = {s for s in nm(TOPO_LIB, "--defined-only") if s.startswith("topology_")}
    assert TOPOLOGY_API <= defined
    assert defined - TOPOLOGY_API == {"topology_shd_getPathPacketCount"}
    assert {"schedulerpolicygpurounds_new", "schedulerpolicygpurounds_new_bridged",
            "schedulerpolicygpurounds_error"} <= nm(TOPO_LIB, "--defined-only")
    undefined = nm(TOPO_LIB, "--undefined-only")
    assert SHADOW_PROVIDES <= undefined


@pytest.mark.skipif(not have_reference(), reason="reference tree / conda glib headers absent")
def test_topology_header_declares_exactly_the_adapted_functions():
    h = open(os.path.join(REF, "main", "routing", "topology.h")).read()
    assert set(re.findall(r"\b(topology_[A-Za-z]+)\(", h)) == TOPOLOGY_API


@pytest.mark.skipif(not have_reference() or not shutil.which("gcc"), reason="reference tree absent")
def test_topology_adapter_compiles_against_the_reference_header(tmp_path):
    cmd = ["gcc", "-std=gnu11", "-D_GNU_SOURCE", "-fsyntax-only", "-Werror", "-Wall", "-Wno-unused-function",
           "-include", os.path.join(REF, "main", "routing", "topology.h"), "-I" + REF] + GLIB + \
          [os.path.join(PKG, "host", "topology_shd.c")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(not have_reference() or not shutil.which("gcc"), reason="reference tree absent")
def test_policy_adapter_compiles_against_the_reference_header():
    src = os.path.join(PKG, "host", "sched_policy_shd.c")
    cmd = ["gcc", "-std=gnu11", "-D_GNU_SOURCE", "-fsyntax-only", "-Werror", "-Wall", "-Wno-unused-function",
           "-DSHD_CHECK_AGAINST_REFERENCE", "-include",
           os.path.join(REF, "main", "core", "scheduler", "scheduler_policy.h"), "-I" + REF] + GLIB + [src]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
