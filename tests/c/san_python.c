/*
 * san_python.c -- a Python interpreter linked against the AddressSanitizer runtime, so that the
 * sanitizer-instrumented host libraries (ompi-release_amd/lib_san, Makefile.san) can be loaded by
 * the ctypes-based boundary tests: ASan's runtime must be in the initial library list, which an
 * instrumented executable gives without preloading anything.  CPU only (tools/san_boundary.sh).
 */
#include <Python.h>

int main(int argc, char **argv) { return Py_BytesMain(argc, argv); }
