"""Package metadata: the ``mopo`` console command (the reference's setup.py:14-18 entry point) maps to
mopo_amd.__main__:main.  libmopo_hip.so is built in-tree first (``make -C mopo_amd/csrc``) and shipped
as package data."""
from setuptools import find_packages, setup

setup(
    name='mopo_amd',
    version='0.2.0',
    packages=find_packages(include=['mopo_amd', 'mopo_amd.*']),
    package_data={'mopo_amd': ['libmopo_hip.so']},
    entry_points={'console_scripts': ['mopo=mopo_amd.__main__:main']},
    python_requires='>=3.8',
)
