import os
for f in os.environ["COMBO"].split(","):
    exec(open("tools/patches/" + f + ".py").read())
