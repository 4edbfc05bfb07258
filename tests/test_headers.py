"""The public headers compile on their own with strict warnings as errors: include/chunky_ec.h as
C99 and C++17 (the C-ABI a cgo / bindgen / JNI shim would consume), include/chunky_ec.hpp as
C++17 and C++20 (the host layer).  Syntax-only, no GPU and no library needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def _compile(compiler, std, lang, src, tmp_path):
    if not shutil.which(compiler):
        pytest.skip(f"{compiler} not available")
    f = tmp_path / ("t.c" if lang == "c" else "t.cpp")
    f.write_text(src)
    r = subprocess.run([compiler, f"-std={std}", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                        "-I", INC, str(f)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("std", ["c99", "c11"])
def test_c_header_as_c(tmp_path, std):
    _compile("gcc", std, "c", '#include "chunky_ec.h"\nint main(void) { return 0; }\n', tmp_path)


def test_c_header_as_cpp(tmp_path):
    _compile("g++", "c++17", "cpp", '#include "chunky_ec.h"\nint main() { return 0; }\n', tmp_path)


@pytest.mark.parametrize("std", ["c++17", "c++20"])
def test_host_layer_header(tmp_path, std):
    src = ('#include "chunky_ec.hpp"\n'
           'int main() {\n'
           '    chunky_ec::FileWriteBuilder b;\n'
           '    b.chunk_size(1 << 20).data_chunks(10).parity_chunks(4);\n'
           '    chunky_ec::release_thread_buffers();\n'
           '    return 0;\n'
           '}\n')
    _compile("g++", std, "cpp", src, tmp_path)
