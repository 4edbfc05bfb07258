// Links libchunky_ec.so built by `make -C chunky-bits_amd/csrc` (or the path in CHUNKY_EC_LIB_DIR).
use std::env;
use std::path::PathBuf;

fn main() {
    let dir = env::var("CHUNKY_EC_LIB_DIR").map(PathBuf::from).unwrap_or_else(|_| {
        PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../../chunky_ec")
    });
    println!("cargo:rerun-if-env-changed=CHUNKY_EC_LIB_DIR");
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=chunky_ec");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
}
