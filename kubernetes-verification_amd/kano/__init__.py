"""kano -- MI355X-native drop-in for kano_py's ``kano`` package.

Modules mirror the reference: ``kano.model`` (data model and the device-resident
ReachabilityMatrix), ``kano.algorithm`` (the Kano checks) and ``kano.parser``
(YAML front-end).  Put the directory holding this package on ``sys.path`` and
``from kano.model import *`` works as with kano_py.
"""
__version__ = "0.1.0"
