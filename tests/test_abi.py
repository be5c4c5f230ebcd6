"""The C-ABI library loads and exports exactly what include/shdgpu.h declares
(no compute calls: runs on CPU)."""
import os
import re
import subprocess

import shdgpu as S

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    out = set()
    for name in ("shdgpu.h", "shdtcp.h"):   # the library's C ABI (include/*.h)
        h = open(os.path.join(REPO, "include", name)).read()
        out |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(shd_[a-z_0-9]+)\(", h, re.M))
    return out


def exported(path=None):
    out = subprocess.run(["nm", "-D", "--defined-only", path or S.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("shd_")}


def test_library_loads(shd):
    assert b"gfx950" in shd.lib().shd_version()


def test_every_declared_symbol_is_exported_and_bound():
    d, e = declared(), exported()
    assert d, "no declarations parsed"
    assert d == e, (d - e, e - d)
    assert d == set(S.exported_symbols())


def test_test_hook_build_exports_the_same_abi():
    # tests/hook_worker.py and xgroup_worker.py load the test build in place of
    # the product library: it must bind every symbol shdgpu.lib() binds
    th = os.path.join(os.path.dirname(S.LIB_PATH), "libshdgpu_th.so")
    assert exported(th) == exported()


def test_code_object_targets_gfx950():
    blob = open(S.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"sm_"):
        assert other not in blob


def test_no_oracle_on_product_path():
    # the product library never links or embeds the oracle
    out = subprocess.run(["nm", "-D", S.LIB_PATH], capture_output=True, text=True).stdout
    assert " o_" not in out
    ldd = subprocess.run(["ldd", S.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in ldd
    for root, _, files in os.walk(os.path.join(REPO, "shadow-1_amd")):
        for f in files:
            if f.endswith((".py", ".c", ".h", ".hip", ".cpp")):
                src = open(os.path.join(root, f), errors="ignore").read()
                assert "oracle_ffi" not in src and "liboracle" not in src, f


def test_no_kernel_uses_a_dynamic_stack():
    # a recursive or indirect device call makes the compiler under-size a
    # lane's scratch (the runtime then allocates the static estimate only);
    # every kernel's AMDGPU metadata must say its stack size is exact
    import re
    blob = open(S.LIB_PATH, "rb").read()
    key = b".uses_dynamic_stack"
    vals = [blob[m.end():m.end() + 1] for m in re.finditer(re.escape(key), blob)]
    assert vals, "no kernel metadata found"
    assert set(vals) == {b"\xc2"}, "a kernel uses a dynamic stack (msgpack true)"


def test_tcp_struct_layout_matches_the_header(tmp_path):
    # the ctypes mirrors of shd_tcp_model / shd_tcp_result against gcc's layout
    import ctypes as C
    src = tmp_path / "l.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s/include/shdtcp.h"\n'
                   'int main(void){printf("%%zu %%zu %%zu %%zu %%zu\\n", sizeof(shd_tcp_model),'
                   ' offsetof(shd_tcp_model, host_vertex), offsetof(shd_tcp_model, packets_per_host),'
                   ' sizeof(shd_tcp_result), offsetof(shd_tcp_result, deliveries));'
                   'printf("%%zu %%zu\\n", offsetof(shd_tcp_model, path_cache),'
                   ' offsetof(shd_tcp_result, max_round_deliveries));return 0;}\n' % REPO)
    exe = tmp_path / "l"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(S.TcpModel), S.TcpModel.host_vertex.offset, S.TcpModel.packets_per_host.offset,
                   C.sizeof(S.TcpResult), S.TcpResult.deliveries.offset, S.TcpModel.path_cache.offset,
                   S.TcpResult.max_round_deliveries.offset]


def test_model_struct_layout_matches_the_header(tmp_path):
    # the ctypes mirrors of shd_model / shd_udp_app / shd_run_stats against gcc's layout
    import ctypes as C
    src = tmp_path / "m.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s/include/shdgpu.h"\n'
                   'int main(void){printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(shd_model),'
                   ' offsetof(shd_model, app_peer), offsetof(shd_model, app_spec), offsetof(shd_model, host_app),'
                   ' offsetof(shd_model, n_app_specs), sizeof(shd_udp_app), sizeof(shd_run_stats));'
                   'printf("%%zu\\n", offsetof(shd_run_stats, n_rounds_replayed));return 0;}\n' % REPO)
    exe = tmp_path / "m"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(S.Model), S.Model.app_peer.offset, S.Model.app_spec.offset, S.Model.host_app.offset,
                   S.Model.n_app_specs.offset, C.sizeof(S.UdpApp), C.sizeof(S.RunStats),
                   S.RunStats.n_rounds_replayed.offset]


def test_pc_info_layout_matches_the_header(tmp_path):
    # the ctypes mirror of shd_pc_info (round 6 added n_tie_rows_predicted) against gcc's layout
    import ctypes as C
    src = tmp_path / "p.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s/include/shdgpu.h"\n'
                   'int main(void){printf("%%zu %%zu %%zu %%zu\\n", sizeof(shd_pc_info),'
                   ' offsetof(shd_pc_info, n_tie_rows), offsetof(shd_pc_info, n_tie_rows_global),'
                   ' offsetof(shd_pc_info, n_tie_rows_predicted));return 0;}\n' % REPO)
    exe = tmp_path / "p"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(S.PcInfo), S.PcInfo.n_tie_rows.offset, S.PcInfo.n_tie_rows_global.offset,
                   S.PcInfo.n_tie_rows_predicted.offset]
