"""The Java (Panama) binding in wireguard-java_amd/java binds libwgaead symbols that exist in
include/wgaead.h with the header's arity and 64-bit-ness (no JDK in the image, so this is a
source-level check of WgAead.java's FunctionDescriptors against the C prototypes)."""
import os
import re

from wgtest import ROOT

HDR = open(os.path.join(ROOT, "include", "wgaead.h")).read()
JAVA = open(os.path.join(ROOT, "wireguard-java_amd", "java", "ax", "xz", "wireguard", "noise", "crypto",
                         "WgAead.java")).read()


def _prototypes():
    body = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|void\*|const char\*)\s+(wg_\w+)\s*\(([^)]*)\)\s*;", body, re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = args
    return out


def _c_kind(arg: str) -> str:
    a = re.sub(r"/\*.*?\*/", "", arg).strip()
    if "*" in a:
        return "ADDRESS"
    if "uint64_t" in a:
        return "JAVA_LONG"
    return "JAVA_INT"


def test_every_java_downcall_matches_the_header():
    protos = _prototypes()
    calls = re.findall(r'down\(linker, symbols, "(wg_\w+)",\s*FunctionDescriptor\.of\(([^;]*?)\)\);', JAVA, re.S)
    assert len(calls) >= 20
    for name, desc in calls:
        assert name in protos, f"{name} bound in WgAead.java but not declared in wgaead.h"
        kinds = [k.strip() for k in desc.replace("\n", " ").split(",")]
        args = kinds[1:]  # first is the return layout
        want = [_c_kind(a) for a in protos[name]]
        assert args == want, (name, args, want)


def test_java_no_key_code_matches_the_header():
    """WgAead.check turns WG_ENOKEY (a cleaned or never-set key slot) into IllegalStateException, as the
    reference's closed key arena does; the constant must be the header's."""
    c = int(re.search(r"#define WG_ENOKEY \((-\d+)\)", HDR).group(1))
    j = int(re.search(r"static final int WG_ENOKEY = (-\d+);", JAVA).group(1))
    assert c == j
    assert "throw new IllegalStateException" in JAVA
