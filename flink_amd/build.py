"""Build libflinkgpu.so in-tree (hipcc, gfx950) with flink_amd/Makefile."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def build(jobs: int = 4) -> str:
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", HERE], check=True)
    return os.path.join(HERE, "libflinkgpu.so")


if __name__ == "__main__":
    print(build())
