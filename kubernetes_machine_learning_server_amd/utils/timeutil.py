"""Wall-clock helpers with the reference's formats."""
from __future__ import annotations

from datetime import datetime, timezone

TZ_NAME = "America/Sao_Paulo"
FMT = "%Y-%m-%d %H:%M:%S"


def current_time_str(now: "datetime | None" = None) -> str:
    """Sao Paulo local time ``YYYY-MM-DD HH:MM:SS`` (``machine-learning/main.py:414-418``)."""
    now = now or datetime.now(timezone.utc)
    try:
        import pytz
        tz = pytz.timezone(TZ_NAME)
    except Exception:  # pragma: no cover
        from zoneinfo import ZoneInfo
        tz = ZoneInfo(TZ_NAME)
    return now.astimezone(tz).strftime(FMT)


def format_timedelta(seconds: float) -> str:
    """pandas ``Timedelta`` str format, e.g. ``0 days 00:00:20.313968`` (main.py:308)."""
    import pandas as pd
    return str(pd.Timedelta(seconds=seconds))
