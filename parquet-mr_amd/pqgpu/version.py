"""created_by -> whether DELTA_BYTE_ARRAY pages need the PARQUET-246 carry-over (host metadata).

Restates parquet-mr's CorruptDeltaByteArrays.requiresSequentialReads
(parquet-column/src/main/java/org/apache/parquet/CorruptDeltaByteArrays.java:31-84) over
VersionParser.parse (parquet-common/src/main/java/org/apache/parquet/VersionParser.java, FORMAT) and
SemanticVersion.parse / compareTo (parquet-common/.../SemanticVersion.java:39-160). A True answer means
the chunk's DELTA_BYTE_ARRAY pages after its first are flagged PQG_PAGE_DBA_CARRY
(batch.ColumnChunk.dba_carry)."""
import re

from . import abi

# VersionParser.FORMAT: "(.*?)\\s+version\\s*(?:([^(]*?)\\s*(?:\\(\\s*build\\s*([^)]*?)\\s*\\))?)?"
_CREATED_BY = re.compile(r"(.*?)\s+version\s*(?:([^(]*?)\s*(?:\(\s*build\s*([^)]*?)\s*\))?)?")
# SemanticVersion.FORMAT: major.minor.patch, unknown, -prerelease, +build
_SEMVER = re.compile(r"^(\d+)\.(\d+)\.(\d+)([^-+]*)?(?:-([^+]*))?(?:\+(.*))?$")
_FIXED = (1, 8, 0)  # PARQUET_246_FIXED_VERSION


def parse_created_by(created_by):
    """VersionParser.parse: (application, version, build hash); ValueError if it does not match."""
    m = _CREATED_BY.fullmatch(created_by)
    if not m or not m.group(1):
        raise ValueError(f"Could not parse created_by: {created_by}")
    return m.group(1), (m.group(2) or None), (m.group(3) or None)


def semver_before_fixed(version):
    """SemanticVersion.parse(version).compareTo(1.8.0) < 0; None when it does not parse."""
    if version is None:
        return None
    m = _SEMVER.fullmatch(version)
    if not m:
        return None
    try:
        mmp = tuple(int(g) for g in m.group(1, 2, 3))
    except ValueError:
        return None
    if any(x > 2**31 - 1 for x in mmp):  # Integer.parseInt overflow -> SemanticVersionParseException
        return None
    if mmp != _FIXED:
        return mmp < _FIXED
    # equal numbers: an "unknown" part (prerelease flag) or a -prerelease sorts before the release
    return bool(m.group(4)) or m.group(5) is not None


def requires_sequential_reads(created_by, encoding=abi.DELTA_BYTE_ARRAY):
    """CorruptDeltaByteArrays.requiresSequentialReads(String createdBy, Encoding)."""
    if encoding != abi.DELTA_BYTE_ARRAY:
        return False
    if not created_by:
        return True  # "file version is empty"
    try:
        app, version, _ = parse_created_by(created_by)
    except ValueError:
        return True  # created_by could not be parsed
    if app != "parquet-mr":
        return False  # other applications do not have the bug
    before = semver_before_fixed(version)
    return True if before is None else before
