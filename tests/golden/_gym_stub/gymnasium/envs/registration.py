def register(**kwargs):
    pass
