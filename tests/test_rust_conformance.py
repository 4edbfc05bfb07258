"""The Rust FFI crate (chunky-bits_amd/rust/chunky-ec-sys) against the C header it binds.

There is no cargo in this image, so the crate is never compiled here; this is the check that is
possible: the `extern "C"` block of src/lib.rs and include/chunky_ec.h must declare the same
functions, with the same arity, and every parameter / return type must match in kind (pointer
depth and constness, integer width and signedness); the `cec_part_batch` layout and the ABI
constants must agree too.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "chunky_ec.h")
RUST = os.path.join(ROOT, "chunky-bits_amd", "rust", "chunky-ec-sys", "src", "lib.rs")

# C base type -> canonical name shared with Rust
C_BASE = {"size_t": "usize", "int": "c_int", "unsigned": "c_uint", "unsigned int": "c_uint",
          "uint64_t": "u64", "uint8_t": "u8", "int32_t": "i32", "char": "c_char", "void": "c_void",
          "cec_codec": "cec_codec", "cec_pipeline": "cec_pipeline",
          "cec_read_pipeline": "cec_read_pipeline", "cec_multi": "cec_multi",
          "cec_part_batch": "cec_part_batch", "cec_read_submit": "cec_read_submit",
          "cec_multi_stats": "cec_multi_stats"}


def _strip_c_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def c_type(decl: str, has_name: bool = True):
    """Canonical type of a C declarator like 'const uint8_t* const* data'."""
    toks = re.findall(r"[A-Za-z_][A-Za-z_0-9]*|\*", decl)
    type_words = {w for k in C_BASE for w in k.split()} | {"const"}
    if has_name and toks and toks[-1] != "*" and toks[-1] not in type_words:
        toks = toks[:-1]  # the parameter name
    base_words, consts, stars = [], [False], 0
    cur_const = False
    for tk in toks:
        if tk == "const":
            cur_const = True
        elif tk == "*":
            consts[-1] = consts[-1] or cur_const
            consts.append(False)
            cur_const = False
            stars += 1
        else:
            base_words.append(tk)
    consts[-1] = consts[-1] or cur_const
    base = C_BASE[" ".join(base_words)]
    # consts[0]: const of the base; consts[i]: const of pointer level i (the pointee of i+1)
    t = base
    pointee_const = consts[0]
    for level in range(stars):
        t = ("ptr", pointee_const, t)
        pointee_const = consts[level + 1]
    return t


def rust_type(s: str):
    s = s.strip()
    m = re.match(r"\*(const|mut)\s+(.*)$", s)
    if m:
        return ("ptr", m.group(1) == "const", rust_type(m.group(2)))
    return s.split("::")[-1].strip()


def header_functions():
    src = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z_0-9 \*]*?)\b(cec_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src):
        ret, name, params = m.group(1).strip(), m.group(2), m.group(3).strip()
        if name.startswith("cec_") and ret.startswith("typedef"):
            continue
        ps = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
        out[name] = (c_type(ret, has_name=False), [c_type(p) for p in ps])
    return out


def rust_functions():
    src = open(RUST).read()
    block = re.search(r'extern "C"\s*\{(.*?)\n    \}', src, flags=re.S).group(1)
    block = re.sub(r"//[^\n]*", "", block)
    out = {}
    for m in re.finditer(r"pub fn (cec_[a-z0-9_]+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", block,
                         flags=re.S):
        name, params, ret = m.group(1), m.group(2), m.group(4)
        ps = [p.strip() for p in params.split(",") if p.strip()]
        types = [rust_type(p.split(":", 1)[1]) for p in ps]
        out[name] = (rust_type(ret) if ret else "c_void", types)
    return out


def test_rust_declares_every_header_function_with_matching_types():
    h, r = header_functions(), rust_functions()
    assert len(h) > 60
    assert sorted(h) == sorted(r), (sorted(set(h) - set(r)), sorted(set(r) - set(h)))
    for name in h:
        hret, hps = h[name]
        rret, rps = r[name]
        assert len(hps) == len(rps), name
        assert hret == rret, (name, hret, rret)
        for i, (a, b) in enumerate(zip(hps, rps)):
            assert a == b, (name, i, a, b)


def test_part_batch_layout_and_constants_match():
    hsrc = _strip_c_comments(open(HEADER).read())
    rsrc = open(RUST).read()
    for struct in ("cec_part_batch", "cec_read_submit", "cec_multi_stats"):
        cfields = re.search(rf"typedef struct {struct} \{{(.*?)\}}", hsrc, flags=re.S).group(1)
        cf = [(c_type(f.strip()), f.strip().split()[-1].lstrip("*")) for f in cfields.split(";")
              if f.strip()]
        rfields = re.search(rf"pub struct {struct} \{{(.*?)\}}", rsrc, flags=re.S).group(1)
        rf = [(rust_type(f.split(":", 1)[1]), f.split(":", 1)[0].replace("pub", "").strip())
              for f in rfields.split(",") if ":" in f]
        assert [(t, n) for t, n in cf] == [(t, n) for t, n in rf], struct
    for const in ("CEC_ABI_VERSION", "CEC_READ_REBUILT_ONLY", "CEC_PIPE_EXTERNAL",
                  "CEC_PRESENT_VERIFIED", "CEC_READ_RESILVER", "CEC_READ_VERIFY_ONLY",
                  "CEC_READ_CARRY", "CEC_SUBMIT_PACKED", "CEC_MULTI_WRITE", "CEC_MULTI_READ",
                  "CEC_MULTI_AHEAD"):
        cv = re.search(rf"#define {const}\s+(0x[0-9a-fA-F]+|\d+)u?", hsrc).group(1)
        rv = re.search(rf"pub const {const}:[^=]+=\s*(0x[0-9a-fA-F]+|\d+);", rsrc).group(1)
        assert int(cv, 0) == int(rv, 0), const


def test_status_codes_match_the_crate_mapping():
    """check() in lib.rs maps 1..13 onto reed_solomon_erasure::Error in the header's order."""
    hsrc = _strip_c_comments(open(HEADER).read())
    rsrc = open(RUST).read()
    names = dict((int(v), k) for k, v in re.findall(r"CEC_([A-Z_]+)\s*=\s*(\d+)", hsrc))
    for code, variant in re.findall(r"(\d+) => Error::(\w+),", rsrc):
        camel = "".join(w.capitalize() for w in names[int(code)].split("_"))
        assert camel == variant, (code, camel, variant)


def _crate_sources():
    src_dir = os.path.dirname(RUST)
    return {n: open(os.path.join(src_dir, n)).read() for n in sorted(os.listdir(src_dir))
            if n.endswith(".rs")}


def test_no_panics_on_engine_errors():
    for name, src in _crate_sources().items():
        code = re.sub(r"//[^\n]*", "", src)
        assert "panic!" not in code and ".expect(" not in code and ".unwrap()" not in code, name


def test_every_ffi_use_is_declared():
    """Every sys::cec_* call in the crate (lib.rs wrappers, batch.rs's BatchWriter) names a
    function of the extern block (hence of the header, by the test above)."""
    declared = set(rust_functions())
    for name, src in _crate_sources().items():
        used = set(re.findall(r"sys::(cec_[a-z0-9_]+)\s*\(", src))
        assert used <= declared, (name, sorted(used - declared))
    batch = _crate_sources()["batch.rs"]
    assert "pub mod batch;" in open(RUST).read()
    # the batched writer goes through the asynchronous scheduler calls and part_encode
    for call in ("submit_encode_hash", ".wait(", "part_encode(", "HostBuffer::zeroed"):
        assert call in batch, call


def test_batch_writer_mirrors_the_cpp_loop():
    """BatchWriter::write is the C++ FileWriteBuilder::write_full_parts loop plus the reader
    (writer.rs:172-194): two windows alternating, the older one collected first, the short last
    part through part_encode; the C++ loop is the one the GPU tests run."""
    batch = _crate_sources()["batch.rs"]
    body = batch[batch.index("pub fn write<"):batch.index("fn fill<")]
    order = [body.index(s) for s in ("self.fill(", "self.submit(", "self.collect(prev",
                                      "self.collect(current", "self.short_part(")]
    assert order == sorted(order)
    assert "slot ^= 1" in body
    hpp = open(os.path.join(ROOT, "include", "chunky_ec.hpp")).read()
    assert "write_full_parts" in hpp and "cur ^= 1" in hpp


def test_batch_reader_mirrors_the_cpp_and_python_loops():
    """BatchReader::read is the C++ read_run / retry_start / retry_collect loop (and
    chunky_ec/batchreader.py, its GPU-tested Python twin): per step every window is polled
    (checked once its job is done, its retry's next round queued once the last one is), the
    oldest finished and handed out (loaded data chunks from the window's chunk buffer,
    REBUILT_ONLY), then the next window loaded and submitted into its buffers; failed parts
    retried with PRESENT_VERIFIED chunks plus untried ones until they decode,
    TooFewShardsPresent when none is left."""
    batch = _crate_sources()["batch.rs"]
    body = batch[batch.index("pub fn read<"):batch.index("    fn load<")]
    order = [body.index(s) for s in ("self.poll(live, i + 1", "self.finish(&mut w", "self.load(",
                                      "self.submit(")]
    assert order == sorted(order) and "self.drain(&live)" in body
    assert "read_windows_for(depth)" in batch and "self.multi.query(" in batch
    assert "CEC_READ_REBUILT_ONLY" in open(RUST).read() and "window_slice(ch, p, l)" in batch
    retry = batch[batch.index("    fn retry_start<"):batch.index("    fn drain(&self, live: &[Option<LiveRead>])")]
    for s in ("CEC_PRESENT_VERIFIED", "have + added < d", "TooFewShardsPresent",
              "self.multi.submit_read_carry(", "self.multi.wait(rt.job)"):
        assert s in retry, s
    drain = batch[batch.index("    fn drain(&self, live: &[Option<LiveRead>])"):]
    drain = drain[:drain.index("\n    }\n")]
    assert "carry_release(" in drain and "rt.cid" in drain and "self.multi.wait(rt.job)" in drain
    # a round in flight when the read fails: its ids for parts still short of d go back too
    # (the leak tests/cpp/host_loop_fuzz.cpp and test_batch_reader_polling_loop_fuzz found)
    assert "rt.r_cout.iter().take(rt.g)" in drain
    # range reads (FileReadBuilder::seek / take): the same part selection and trimming as the C++
    # FileReadBuilder and the Python FileReader.read_range
    rr = batch[batch.index("    pub fn read_range<"):batch.index("    pub fn read_parts<")]
    for s in ("range_len(length, seek, take)", "skip >= part_len(first)", "covered < skip + want",
              "self.read_parts(shapes, digests, first, end,"):
        assert s in rr, s
    assert "pub fn range_len(length: u64, seek: u64, take: u64) -> u64" in batch
    py = open(os.path.join(ROOT, "chunky-bits_amd", "chunky_ec", "batchreader.py")).read()
    for s in ("def _load", "def _submit", "def _check", "def _poll", "def _finish",
              "def _retry_start", "def _retry_round", "def _retry_collect", "have + added < d",
              "PRESENT_VERIFIED", "TOO_FEW_SHARDS_PRESENT"):
        assert s in py, s


def test_location_walk_is_the_same_rule_in_rust_python_and_cpp():
    """The read loops walk a chunk's locations before drawing another chunk (file_part.rs:100-107)
    and verify / resilver hash every location (:236-243, :277-289), resilver appending the
    rebuilt copy's location (:346): the same helpers and steps in the Rust crate, its Python twins
    (run on the GPU) and the C++ host layer (run on the GPU by the mirror test)."""
    batch = _crate_sources()["batch.rs"]
    for s in ("fn next_copy<", "fn draw_order(", "FnMut(usize, usize, usize) -> Option<(usize, Vec<u8>)>",
              "pub fn read_part<", "pub struct FileReader", "pub struct BatchChecker",
              "pub struct FileChecker", "CEC_PRESENT_VERIFIED", "submit_verify(", "submit_resilver(",
              "pub enum CopyCheck"):
        assert s in batch, s
    retry = batch[batch.index("    fn retry_start<"):batch.index("    fn drain(&self, live: &[Option<LiveRead>])")]
    assert "draw_order(" in retry and "next_copy(" in retry and "cursor[x]" in retry
    lib = open(RUST).read()
    for s in ("pub fn sha256_many(", "pub unsafe fn submit_verify(", "pub unsafe fn submit_resilver(",
              "pub fn build_id("):
        assert s in lib, s
    py_reader = open(os.path.join(ROOT, "chunky-bits_amd", "chunky_ec", "batchreader.py")).read()
    for s in ("def next_copy", "def draw_order", "def read_part", "class FileReader"):
        assert s in py_reader, s
    py_check = open(os.path.join(ROOT, "chunky-bits_amd", "chunky_ec", "batchcheck.py")).read()
    for s in ("class BatchChecker", "class FileChecker", "PRESENT_VERIFIED", "def _submit_resilver",
              "def _submit_verify"):
        assert s in py_check, s
    hpp = open(os.path.join(ROOT, "include", "chunky_ec.hpp")).read()
    for s in ("inline const Bytes* next_copy(", "inline std::vector<size_t> draw_order(",
              "std::vector<Location> locations;", "c.locations.push_back(dest.write_shard(",
              "CEC_PRESENT_VERIFIED"):
        assert s in hpp, s
