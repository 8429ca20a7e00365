"""Packaging (reference: python/setup.py + build.sh, which build the JVM jars with Maven and
copy them into the wheel). Here ``build_ext`` compiles the native runtime, services and the
gfx950 HIP kernels in place (raydp_amd/native/build.py), and the wheel carries them.

    pip install --no-build-isolation .        # or: python setup.py build_ext --inplace
"""
import os

from setuptools import Command, find_packages, setup
from setuptools.command.build_py import build_py

ROOT = os.path.dirname(os.path.abspath(__file__))


class BuildNative(Command):
    description = "compile the native runtime, services and gfx950 HIP kernels in place"
    user_options = [("force", "f", "rebuild everything")]

    def initialize_options(self):
        self.force = False

    def finalize_options(self):
        pass

    def run(self):
        import sys
        sys.path.insert(0, ROOT)
        os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
        from raydp_amd.native import build
        build.build_all(force=bool(self.force))


class BuildPyWithNative(build_py):
    def run(self):
        self.run_command("build_native")
        super().run()


setup(
    name="raydp-amd",
    version="1.7.0.dev0",
    description="Spark-on-Ray data + training engine with RayDP's API, native to AMD MI355X",
    packages=find_packages(include=["raydp", "raydp.*", "raydp_amd", "raydp_amd.*"]),
    package_data={"raydp_amd.native": ["*.so", "raydp_supervisor", "raydp_appmaster", "raydp_shuffle_service"],
                  "raydp_amd.mpi": ["*.proto"]},
    include_package_data=True,
    python_requires=">=3.9",
    install_requires=["numpy", "pandas", "psutil", "pyarrow>=4.0.1", "cloudpickle", "protobuf", "grpcio", "torch"],
    entry_points={"console_scripts": ["raydp-submit=raydp_amd.submit:main"]},
    cmdclass={"build_native": BuildNative, "build_py": BuildPyWithNative},
)
