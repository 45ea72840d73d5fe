// Compiles the engine's HIP sources with hipcc for gfx950 and links the resulting shared library:
// the same translation units, common flags and per-unit flags as ggrs_amd/build.py (UNITS, FLAGS,
// UNIT_FLAGS), so the crate links the library bench.py measures (tests/test_rust_ffi.py pins both).
use std::path::PathBuf;
use std::process::Command;

// ggrs_amd/build.py FLAGS
const FLAGS: &[&str] = &[
    "-O3",
    "--offload-arch=gfx950",
    "-ffp-contract=off",
    "-fPIC",
    "-std=c++17",
    "-Wall",
    "-Wno-unused-function",
];
// ggrs_amd/build.py ILP: LLVM's max-ilp machine scheduler for the one-wave-per-SIMD step kernels
const ILP: &[&str] = &["-mllvm", "-amdgpu-sched-strategy=max-ilp"];
const NONE: &[&str] = &[];
// ggrs_amd/build.py UNITS with UNIT_FLAGS
const UNITS: &[(&str, &[&str])] = &[
    ("engine.hip", ILP),
    ("requests.hip", NONE),
    ("branch.hip", NONE),
    ("particles.hip", NONE),
    ("p2p.hip", ILP),
    ("p2p_sched.hip", ILP),
    ("codec.hip", NONE),
    ("lane_encode.cpp", NONE),
];

fn main() {
    let out = PathBuf::from(std::env::var("OUT_DIR").unwrap());
    let root = PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap()).join("../..");
    let csrc = root.join("ggrs_amd/csrc");
    let hipcc = std::env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let mut objs = Vec::new();
    for (unit, unit_flags) in UNITS {
        let obj = out.join(format!("{unit}.o"));
        let status = Command::new(&hipcc)
            .args(FLAGS)
            .args(*unit_flags)
            .arg("-I").arg(root.join("include"))
            .arg("-I").arg(&csrc)
            .arg("-c").arg("-o").arg(&obj)
            .arg(csrc.join(unit))
            .status()
            .expect("hipcc not found");
        assert!(status.success(), "hipcc failed on {unit}");
        objs.push(obj);
    }
    let lib = out.join("libggrs_amd.so");
    let status = Command::new(&hipcc)
        .args(["--offload-arch=gfx950", "-shared", "-fPIC", "-o"])
        .arg(&lib)
        .args(&objs)
        .status()
        .expect("hipcc not found");
    assert!(status.success(), "hipcc link failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=ggrs_amd");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", out.display());
    println!("cargo:rerun-if-changed={}", csrc.display());
    println!("cargo:rerun-if-changed={}", root.join("include/ggrs_amd.h").display());
}
