def register(*a, **k):
    return None
