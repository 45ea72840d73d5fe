// Compiles the engine's HIP sources with hipcc for gfx950 and links the resulting shared library.
use std::path::PathBuf;
use std::process::Command;

fn main() {
    let out = PathBuf::from(std::env::var("OUT_DIR").unwrap());
    let root = PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap()).join("../..");
    let csrc = root.join("ggrs_amd/csrc");
    let hipcc = std::env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let lib = out.join("libggrs_amd.so");
    let status = Command::new(hipcc)
        .args(["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC", "-shared", "-std=c++17"])
        .arg("-I").arg(root.join("include"))
        .arg("-I").arg(&csrc)
        .arg("-o").arg(&lib)
        .arg(csrc.join("engine.hip"))
        .arg(csrc.join("requests.hip"))
        .arg(csrc.join("branch.hip"))
        .arg(csrc.join("particles.hip"))
        .arg(csrc.join("p2p.hip"))
        .arg(csrc.join("p2p_sched.hip"))
        .arg(csrc.join("codec.hip"))
        .arg(csrc.join("lane_encode.cpp"))
        .status()
        .expect("hipcc not found");
    assert!(status.success(), "hipcc failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=ggrs_amd");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include/ggrs_amd.h").display());
}
