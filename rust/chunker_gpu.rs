// pbs-datastore/src/chunker_gpu.rs -- drop-in for `pbs_datastore::Chunker`
// (pbs-datastore/src/chunker.rs:18-186, re-exported at pbs-datastore/src/lib.rs:199)
// over the C ABI of include/pbs_chunker.h (libpbschunk.so, built for gfx950).
//
// UNVERIFIED: this image has no Rust toolchain, so this file has never been compiled.
// tests/cpp/shim_sequence.c replays its exact call sequence through the same C ABI
// (new -> scan ... -> free; the not-a-power-of-two panic; a failed scan ->
// last_error -> strerror -> panic -> free) and runs in the GPU test suite
// (tests/test_shim_sequence.py).
//
// Selected in pbs-datastore/src/lib.rs behind a cargo feature:
//
//     #[cfg(feature = "gpu-chunker")]
//     mod chunker_gpu;
//     #[cfg(feature = "gpu-chunker")]
//     pub use chunker_gpu::Chunker;
//     #[cfg(not(feature = "gpu-chunker"))]
//     pub use chunker::Chunker;
//
// The callers -- pbs_client::ChunkStream (pbs-client/src/chunk_stream.rs:40-77),
// DynamicChunkWriter (pbs-datastore/src/dynamic_index.rs:493-515) and the examples --
// use `Chunker::new(usize)` and `Chunker::scan(&mut self, &[u8]) -> usize` unchanged.

use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};

const PBS_ERR_NOT_POW2: c_int = -1; // include/pbs_chunker.h

#[link(name = "pbschunk")]
extern "C" {
    fn pbs_chunker_new(chunk_size_avg: usize, err: *mut c_int) -> *mut c_void;
    fn pbs_chunker_free(c: *mut c_void);
    fn pbs_chunker_scan(c: *mut c_void, data: *const u8, len: usize) -> usize;
    fn pbs_chunker_last_error(c: *const c_void) -> c_int;
    fn pbs_strerror(code: c_int) -> *const c_char;
}

fn strerror(code: c_int) -> String {
    // SAFETY: pbs_strerror returns a static NUL-terminated string for every code
    unsafe { CStr::from_ptr(pbs_strerror(code)) }.to_string_lossy().into_owned()
}

/// Content-defined chunker (Buzhash over a 64-byte window, chunker.rs:18-33), hashed on
/// the GPU.  Same thresholds as the reference: min = avg / 4, max = avg * 4,
/// break when (h & mask) >= mask - 2 (chunker.rs:91-105, :172-186).
pub struct Chunker {
    h: *mut c_void,
}

// One owner at a time, like the reference (`scan` takes `&mut self`); ChunkStream is
// moved into a tokio task (proxmox-backup-client/src/main.rs:206-211), so the handle must
// be Send.  It is not Sync: the C handle is single-owner (include/pbs_chunker.h).
unsafe impl Send for Chunker {}

impl Chunker {
    /// chunker.rs:75-106: panics when `chunk_size_avg` is not a power of two.
    pub fn new(chunk_size_avg: usize) -> Self {
        let mut err: c_int = 0;
        // SAFETY: err is a valid out-pointer; a NULL return is handled below
        let h = unsafe { pbs_chunker_new(chunk_size_avg, &mut err) };
        if h.is_null() {
            if err == PBS_ERR_NOT_POW2 {
                panic!("got unexpected chunk size - not a power of two.");
            }
            panic!("GPU chunker unavailable: {}", strerror(err));
        }
        Self { h }
    }

    /// chunker.rs:112-168: 0 if `data` holds no chunk boundary (all of it consumed into
    /// the state), else the position just after the cut byte, relative to `data`.
    pub fn scan(&mut self, data: &[u8]) -> usize {
        // SAFETY: self.h is a live handle owned by self; data is a valid slice
        let r = unsafe { pbs_chunker_scan(self.h, data.as_ptr(), data.len()) };
        if r == usize::MAX {
            // the reference's scan is infallible: a device error becomes a panic
            // SAFETY: self.h is a live handle
            let code = unsafe { pbs_chunker_last_error(self.h) };
            panic!("GPU chunker failed: {}", strerror(code));
        }
        r
    }
}

impl Drop for Chunker {
    fn drop(&mut self) {
        // SAFETY: self.h came from pbs_chunker_new and is freed exactly once
        unsafe { pbs_chunker_free(self.h) }
    }
}
