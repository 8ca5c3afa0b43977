"""flink-skyline-qos_amd: MI355X-native engine for the skyline hot path of
Asterinos1/Flink-Skyline-QoS.  The importable Python package is `skyline/`
(add this directory to sys.path); the native library is build/libskyline_hip.so."""
