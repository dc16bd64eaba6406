#!/usr/bin/env python
"""Packaging for orange3_spark_amd (engine) + orangecontrib.spark_amd (Orange add-on).

Entry points mirror the reference add-on's (reference setup.py:5-29): widget
categories, tutorials, the add-on registration and widget help.  ``build_py`` compiles
the gfx950 kernel library in-tree first (hipcc; see orange3_spark_amd/ops/build.py).
"""
from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ENTRY_POINTS = {
    "orange.widgets.tutorials": ("sparkamdtutorials = orangecontrib.spark_amd.tutorials",),
    "orange.addons": ("Spark AMD = orangecontrib.spark_amd",),
    "orange.widgets": (
        "Spark Data (AMD) = orangecontrib.spark_amd.widgets.data",
        "Spark ML (AMD) = orangecontrib.spark_amd.widgets.ml",
    ),
    "orange.canvas.help": ("html-index = orangecontrib.spark_amd.widgets:WIDGET_HELP_PATH",),
}


class BuildWithKernels(build_py):
    def run(self):
        from orange3_spark_amd.ops import build as B
        B.build(verbose=True)
        super().run()


setup(
    name="Orange3-Spark-AMD",
    version="0.1.0",
    description="MI355X-native visual-workflow ML backend with Orange3-Spark's widgets and a "
                "Spark-ML-compatible API (gfx950 HIP kernels, RCCL over xGMI)",
    packages=find_packages(include=["orange3_spark_amd*", "orangecontrib*"]),
    package_data={"orange3_spark_amd.ops": ["csrc/*", "_lib/*.so"],
                  "orangecontrib.spark_amd.widgets": ["icons/*.svg"],
                  "orangecontrib.spark_amd.tutorials": ["*.ows"]},
    install_requires=["torch", "numpy", "pandas", "pyarrow", "scipy"],
    extras_require={"orange": ["Orange3"], "test": ["pytest", "scikit-learn"]},
    entry_points=ENTRY_POINTS,
    cmdclass={"build_py": BuildWithKernels},
    python_requires=">=3.10",
    zip_safe=False,
)
