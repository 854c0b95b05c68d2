// CPython launcher built with -fsanitize=<preset> (ray_dynamic_batching_amd/_build.py
// build_sanitized_python): the sanitizer runtime is part of the executable, so it
// is initialised before the interpreter and every extension module -- the
// instrumented _rdb_runtime (RDB_RUNTIME_SO) then runs the Python test suites
// under ThreadSanitizer / AddressSanitizer (tests/test_sanitizers.py).
#include <Python.h>

int main(int argc, char** argv) { return Py_BytesMain(argc, argv); }
