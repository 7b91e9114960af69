"""Dev probe: open a handle through the fake-JVM JNI shim, with torch
imported before the shim's library (argv[1] == "torch"), after it
("late_torch") or not at all; prints the exception message."""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd"), str(ROOT / "tests")]
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch
    print("torch cuda", torch.cuda.is_available())
import test_jni as TJ  # noqa: E402

jvm = TJ.JVM()
if len(sys.argv) > 1 and sys.argv[1] == "late_torch":
    import torch
    print("late torch cuda", torch.cuda.is_available())
h, exc = jvm.call("open", ctypes.c_int64(1000), 2, 3, 0, 0, 0, res=ctypes.c_int64)
print("open ->", h, exc, jvm.L.fj_exception_msg())
