// Builds libcessec.so (HIP kernels for gfx950 + the C ABI) with the repository's Makefile and
// links it. HIPCC / OFFLOAD_ARCH may be overridden from the environment.
use std::env;
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let root = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap()).join("../..");
    let csrc = root.join("cess_amd/csrc");
    let mut make = Command::new("make");
    make.arg("-C").arg(&csrc).arg("../libcessec.so");
    if let Ok(h) = env::var("HIPCC") {
        make.arg(format!("HIPCC={h}"));
    }
    if let Ok(a) = env::var("OFFLOAD_ARCH") {
        make.arg(format!("ARCH={a}"));
    }
    let status = make.status().expect("make (hipcc) for libcessec");
    assert!(status.success(), "building libcessec.so failed");
    let lib_dir = root.join("cess_amd").canonicalize().unwrap();
    println!("cargo:rustc-link-search=native={}", lib_dir.display());
    println!("cargo:rustc-link-lib=dylib=cessec");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", lib_dir.display());
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include/cess_ec.h").display());
}
