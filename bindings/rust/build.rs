// client/build.rs: link libsda_engine.so when the `mi355x` feature is on.  UNCOMPILED (no cargo here).
fn main() {
    if std::env::var_os("CARGO_FEATURE_MI355X").is_some() {
        let dir = std::env::var("SDA_ENGINE_DIR").expect("set SDA_ENGINE_DIR to the directory of libsda_engine.so");
        println!("cargo:rustc-link-search=native={}", dir);
        println!("cargo:rustc-link-lib=dylib=sda_engine");
        println!("cargo:rerun-if-env-changed=SDA_ENGINE_DIR");
    }
}
