"""The C examples of INTEGRATION.md ("Multi-GPU") compile against
include/dips_hip.h as written (C99, every warning an error), so the document
cannot drift from the ABI it describes."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```c\n(.*?)```", text, flags=re.S)


def test_integration_c_example_compiles(tmp_path):
    blocks = _c_blocks()
    assert blocks, "INTEGRATION.md has a C example"
    # the blocks continue one another (the second uses the first's comm)
    body = "\n".join(blocks)
    src = tmp_path / "snippets.c"
    src.write_text(
        "#include <stdint.h>\n#include <stddef.h>\n#include <stdio.h>\n#include \"dips_hip.h\"\n"
        "void example(int rank, int nranks, uint64_t n_total, uint32_t w, uint32_t hgt,\n"
        "             const uint8_t *frames, dips_series_entry *series_local,\n"
        "             dips_series_entry *series_all, uint8_t *out) {\n" + body + "}\n")
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-Wno-unused-variable",
                        "-Wno-unused-parameter", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
