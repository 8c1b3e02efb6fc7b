// pbs-datastore/build.rs lines for the `gpu-chunker` feature (rust/chunker_gpu.rs).
// UNVERIFIED: this image has no Rust toolchain.
//
// PBS_GPU_CHUNKER_LIB: the directory holding libpbschunk.so
// (`make -C proxmox-backup_amd/csrc` builds it there); libamdhip64 comes from ROCm.
fn main() {
    if std::env::var_os("CARGO_FEATURE_GPU_CHUNKER").is_none() {
        return;
    }
    let lib = std::env::var("PBS_GPU_CHUNKER_LIB")
        .unwrap_or_else(|_| "../proxmox-backup_amd/csrc".to_string());
    println!("cargo:rerun-if-env-changed=PBS_GPU_CHUNKER_LIB");
    println!("cargo:rustc-link-search=native={}", lib);
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
    println!("cargo:rustc-link-lib=dylib=pbschunk");
    println!("cargo:rustc-link-lib=dylib=amdhip64");
}
